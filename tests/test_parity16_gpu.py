"""16-bit HIP paths judged against the reference's OWN mixed-precision scheme.

The bar: the oracle run under ``torch.autocast("cuda", dtype)`` on
the same GPU, with the same weights and epsilons — what ``inference/predictors.py:55`` does on
CUDA, and what a bf16 autocast training step of the reference would compute.  The HIP path
must be at least as close to the truth (float64 oracle for gradients, fp32 oracle for the
predictor's statistics) as that scheme, within a stated margin.

* Training step at the BASELINE tile sizes (224 optical / 256 sonar, B=4, N=2) and at 64 px:
  gradients of EVERY parameter tensor (trunks included, 696 tensors) against the float64
  truth, by the per-tensor cosine distribution (median / p10: f16 HIP >= autocast - 0.01 /
  - 0.02; bf16, where both schemes sit at rounding noise (~0.2) at random init, HIP >= autocast
  - NOISE_TENSOR_MARGIN) and each trunk's whole gradient (HIP >= autocast - WEAK_MARGIN, always
  judged: at random init both bf16 schemes sit at cosines 0.08-0.17 and f16 autocast at
  0.004-0.03, so this bar only catches a broken trunk); logits: max |HIP - fp64| <= 2x max
  |autocast - fp64|.
* The same step on a model trained FIT_STEPS steps on the batch (64 px, B = 8 and 32), where
  the reference's scheme resolves the float64 direction: whole-trunk cosines HIP >= autocast -
  COS_MARGIN, with autocast >= RESOLVED asserted (bf16) / HIP >= RESOLVED (f16, whose autocast
  backward underflows) so the bar cannot pass vacuously; the per-tensor
  distribution there at the tight bar (median / p10: HIP >= autocast - 0.01 / - 0.02).
* f16 predictor (the drop-in default path, ``multimodal_predict_and_save``'s maths) at B=64,
  N=8 (64 / 128 px) and B=16, N=8 at 224 / 256 px pooled over PRED_SEEDS fitted models
  (``fit_model``: the class then depends on the input): every item's aleatoric and predictive
  entropy within SURVEY §8c's 1e-2 of the fp32 oracle (or WORST_RATIO x torch-autocast's worst
  item where autocast misses 1e-2 itself), the mean deviations (aleatoric, predictive entropy,
  variance) <= MEAN_RATIO x torch-autocast's, the per-element logit bar missed no more
  often than torch-autocast misses it, argmax agreement >= 99 %.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import bayes_ref, loops_ref
from tests.golden.common import make_batches, SEED_DATA
from tests.helpers import build_pair, EpsBridge, oracle_replay, cosines, fit_model

pytestmark = pytest.mark.gpu

COS_MARGIN = 0.02    # whole-trunk / head gradient cosine: HIP >= autocast - COS_MARGIN
# ... judged where torch-autocast's own whole-trunk cosine is >= RESOLVED.  At random init it
# never is for bf16 (0.08-0.17 over B = 8-32 at 64-224 px, both schemes; f16 autocast 0.004-0.02,
# its backward underflows without a GradScaler; profiles/round5/autocast_resolution_sweep.txt):
# the resolved shapes are a model trained FIT_STEPS fp32 steps on the batch first (bf16: autocast
# 1.000 at B = 8, 0.73-0.76 at B = 32)
RESOLVED = 0.5
FIT_STEPS = 20
RESOLVED_SHAPES = [(64, 64, 8, 2), (64, 64, 32, 2)]   # (S_opt, S_son, B, N)
WEAK_MARGIN = 0.1    # every other shape: HIP >= autocast - WEAK_MARGIN (never skipped)
# per-tensor cosine medians / p10 at random init: ~0.2 for both bf16 schemes, and torch-
# autocast's own median moves 0.215-0.231 from box to box with the vendor kernels it picks
# (profiles/round5: r5a / r4f / round5b logs) — a bar that catches a broken path; the tight
# per-tensor bar (HIP >= autocast - 0.01 median / - 0.02 p10) runs at the resolved shapes
NOISE_TENSOR_MARGIN = 0.05
# f16 predictor (test_predictor_f16_vs_torch_autocast*): SURVEY §8c's 16-bit bars on every item —
# aleatoric and predictive entropy within ENTROPY_BAR of the fp32 oracle, or, on a model where
# the reference's own scheme (the oracle under torch.autocast on the same weights and epsilons)
# misses that bar itself, no more than WORST_RATIO x autocast's worst item (fitted logits span
# +-50; autocast's worst items measured 1.10e-2 / 1.58e-2 / 2.29e-2, profiles/round6) — and the
# mean deviations no more than MEAN_RATIO x autocast's.  At 224 / 256 px the statistics are pooled
# over PRED_SEEDS (data, labels, epsilons, fit) seeds: one seed's mean is one draw of the f16
# rounding noise (round 5's 1.6-2.0x "gap" at seed 0 was: over 8 seeds the two schemes' means are
# 0.98x, per seed 0.55-1.22x — profiles/round6/pred_sweep_centred.log).
# SURVEY's per-element logit bar (5e-2 max(1, |ref|)) is not met by torch-autocast itself on these
# fitted models (144 of 7,168 logits over 8 seeds, |ref| up to 86; this library 86): the bar is
# that the library misses it no more often than autocast does.
ENTROPY_BAR = 1e-2
MEAN_RATIO = 1.25
WORST_RATIO = 1.25
PRED_SEEDS = 4


def _cat_cos(params, truth_params, pick):
    """Cosine of the concatenated gradients of the selected parameters with the truth's."""
    a, t = [], []
    for (n, p), pt in zip(params, truth_params):
        if pick(n) and p.grad is not None and pt.grad is not None:
            a.append(p.grad.detach().double().cpu().flatten())
            t.append(pt.grad.detach().double().cpu().flatten())
    a, t = torch.cat(a), torch.cat(t)
    return float(a @ t / (a.norm() * t.norm()))


def _q(v):
    return float(np.median(v)), float(np.quantile(v, 0.1))


def _cuda(*ts):
    return [t.cuda() for t in ts]


def train_step16_cosines(dt, S_opt, S_son, B, N, truth_device="cpu", fp32_cpu=True, fit_steps=0):
    """One MC training step (N samples, B triplets) of the HIP 16-bit path, of the oracle under
    torch.autocast on the GPU and (fp32_cpu) of the fp32 CPU oracle, with the same weights and
    epsilons; gradients against a float64 run of the oracle (on truth_device).  Returns the
    per-tensor cosines, the whole-gradient cosines of each trunk / the head, and the logit
    errors against float64."""
    from mauv.engine import root_state, set_precision
    from mauv.kl import get_kl_loss
    from mauv import mchead
    o, m = build_pair()
    batch = make_batches(SEED_DATA, 1, B=B, S_opt=S_opt, S_son=S_son)[0]
    x, b, s, y = batch["main_image"], batch["bathy_image"], batch["sss_image"], batch["label"]
    if fit_steps:   # a model trained a few (fp32) steps on this batch, in both implementations
        fit_model(m, *_cuda(x, b, s), y.cuda(), steps=fit_steps)
        o.load_state_dict({k: v.cpu() for k, v in m.state_dict().items()})
    set_precision(m, dt)

    def loss_of(model, dev, dtp=torch.float32, amp=None):
        xs = [t.to(dev, dtp) for t in (x, b, s)]
        if amp is not None:
            with torch.autocast("cuda", dtype=amp):
                lg = torch.stack([model(*xs) for _ in range(N)])
        else:
            lg = torch.stack([model(*xs) for _ in range(N)])
        lg = lg.to(dtp)
        loss = F.cross_entropy(lg.mean(0), y.to(dev)) + bayes_ref.get_kl_loss(model) / B * 0.5
        loss.backward()
        return lg, loss

    # the epsilons depend on the layers only: record them on a 1-triplet 64 px forward
    tiny = make_batches(SEED_DATA, 1, B=1, S_opt=64, S_son=64)[0]
    bridge = EpsBridge(o, m, 99)
    with bridge, torch.no_grad():
        for _ in range(N):
            o(tiny["main_image"], tiny["bathy_image"], tiny["sss_image"])
    bridge.collect()
    o64, (lg64, _) = oracle_replay(o, bridge.store,
                                   lambda mm: loss_of(mm, truth_device, torch.float64),
                                   dtype=torch.float64, device=truth_device)
    oac, (lgac, _) = oracle_replay(o, bridge.store, lambda mm: loss_of(mm, "cuda", amp=dt),
                                   device="cuda")
    root_state(m).eps_provider = bridge.provider
    logits = m.mc_forward(*_cuda(x, b, s), N)
    ce, _, _ = mchead.mc_mean_ce(logits, y.cuda())
    (ce + get_kl_loss(m) / B * 0.5).backward()
    o32 = None
    if fp32_cpu:
        o32, _ = oracle_replay(o, bridge.store, lambda mm: loss_of(mm, "cpu"))
    truth = list(o64.parameters())
    out = {"tensor": {}, "whole": {}}
    out["tensor"]["hip"] = cosines(list(m.named_parameters()), truth)
    out["tensor"]["autocast"] = cosines(list(oac.named_parameters()), truth)
    if o32 is not None:
        out["tensor"]["fp32_cpu"] = cosines(list(o32.named_parameters()), truth)
    for gname in ("image_model_feat", "bathy_model_feat", "sss_model_feat", "head"):
        pick = (lambda n, g=gname: n.startswith(g + ".")) if gname != "head" else \
            (lambda n: not n.split(".")[0].endswith("_feat"))
        out["whole"][gname] = {
            "hip": _cat_cos(list(m.named_parameters()), truth, pick),
            "autocast": _cat_cos(list(oac.named_parameters()), truth, pick),
            "fp32_cpu": None if o32 is None else _cat_cos(list(o32.named_parameters()), truth,
                                                          pick)}
    l64 = lg64.detach().double().cpu()
    out["dlogit_hip"] = (logits.detach().double().cpu() - l64).abs().max().item()
    out["dlogit_autocast"] = (lgac.detach().double().cpu() - l64).abs().max().item()
    return out


def _print_whole(tag, r):
    for gname, c in r["whole"].items():
        f = "" if c["fp32_cpu"] is None else f" (fp32 CPU {c['fp32_cpu']:.5f})"
        print(f"  {tag} {gname:17s} whole-gradient cos vs fp64: HIP {c['hip']:.5f} "
              f"autocast {c['autocast']:.5f}{f}")


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("S_opt,S_son,B,N", [(224, 256, 4, 2), (64, 64, 2, 3)],
                         ids=["224-256", "64"])
def test_train_step16_grads_vs_torch_autocast(dt, S_opt, S_son, B, N):
    r = train_step16_cosines(dt, S_opt, S_son, B, N)
    c_hip, c_ac, c_32 = r["tensor"]["hip"], r["tensor"]["autocast"], r["tensor"]["fp32_cpu"]
    assert set(c_hip) == set(c_ac) and len(c_hip) > 600, len(c_hip)
    names = sorted(c_hip)
    h = np.array([c_hip[n] for n in names])
    a = np.array([c_ac[n] for n in names])
    f = np.array([c_32[n] for n in names])
    trunk = np.array([n.split(".")[0].endswith("_feat") for n in names])
    tag = f"{str(dt)[6:]} {S_opt}/{S_son} B={B} N={N}"
    print(f"\n{tag}: {len(names)} tensors ({trunk.sum()} trunk); per-tensor cos vs fp64 "
          f"median/p10: HIP {_q(h)[0]:.4f}/{_q(h)[1]:.4f} torch-autocast {_q(a)[0]:.4f}/"
          f"{_q(a)[1]:.4f} (fp32 CPU oracle {_q(f)[0]:.4f}/{_q(f)[1]:.4f}); trunk tensors: HIP "
          f"{_q(h[trunk])[0]:.4f}/{_q(h[trunk])[1]:.4f} autocast {_q(a[trunk])[0]:.4f}/"
          f"{_q(a[trunk])[1]:.4f}")
    for sel in (np.ones_like(trunk), trunk):
        (mh, ph), (ma, pa) = _q(h[sel]), _q(a[sel])
        if dt == torch.bfloat16:   # both schemes at rounding noise (docstring of the module)
            assert mh >= ma - NOISE_TENSOR_MARGIN and ph >= pa - NOISE_TENSOR_MARGIN, \
                (mh, ma, ph, pa)
        else:                      # f16: autocast's backward underflows, HIP must resolve more
            assert mh >= ma - 0.01 and ph >= pa - 0.02, (mh, ma, ph, pa)
    _print_whole(tag, r)
    for gname, c in r["whole"].items():
        # at these batches both 16-bit schemes sit near rounding noise for bf16 (cos ~0.1, the
        # BN backward over B = 2-4 per sample amplifies it): a loose bar that still catches a
        # broken trunk; the tight bar is test_train_step16_whole_trunk_resolved's
        assert c["hip"] >= c["autocast"] - WEAK_MARGIN, (gname, c)
    print(f"  max |dlogit| vs fp64: HIP {r['dlogit_hip']:.3e}  torch-autocast "
          f"{r['dlogit_autocast']:.3e}")
    assert r["dlogit_hip"] <= max(2 * r["dlogit_autocast"], 1e-3)


@pytest.mark.parametrize("shape", RESOLVED_SHAPES, ids=lambda s: f"B{s[2]}")
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
def test_train_step16_whole_trunk_resolved(dt, shape):
    """Whole-trunk gradient cosines where the reference's scheme resolves the float64 direction
    (VERDICT r4 next 1), on a model trained FIT_STEPS steps on the batch: bf16 — torch-autocast's
    cosine >= RESOLVED on every trunk (asserted, so the bar is not vacuous) and HIP >= autocast -
    COS_MARGIN; f16 — autocast's training backward does not resolve it (f16 underflow without a
    GradScaler; the reference runs f16 only in its predictor), so HIP's own cosine must be >=
    RESOLVED and >= autocast's - COS_MARGIN.  float64 truth on the GPU."""
    S_opt, S_son, B, N = shape
    r = train_step16_cosines(dt, S_opt, S_son, B, N, truth_device="cuda", fp32_cpu=False,
                             fit_steps=FIT_STEPS)
    tag = f"{str(dt)[6:]} fit={FIT_STEPS} {S_opt}/{S_son} B={B} N={N}"
    print()
    _print_whole(tag, r)
    print(f"  max |dlogit| vs fp64: HIP {r['dlogit_hip']:.3e}  torch-autocast "
          f"{r['dlogit_autocast']:.3e}")
    for gname, c in r["whole"].items():
        if dt == torch.bfloat16:
            assert c["autocast"] >= RESOLVED, (gname, c)
        else:
            assert c["hip"] >= RESOLVED, (gname, c)
        assert c["hip"] >= c["autocast"] - COS_MARGIN, (gname, c)
    assert r["dlogit_hip"] <= max(2 * r["dlogit_autocast"], 1e-3)
    # every parameter tensor: the per-tensor cosine distribution against float64
    c_hip, c_ac = r["tensor"]["hip"], r["tensor"]["autocast"]
    names = sorted(c_hip)
    h = np.array([c_hip[n] for n in names])
    a = np.array([c_ac[n] for n in names])
    print(f"  per-tensor cos vs fp64 median/p10: HIP {_q(h)[0]:.4f}/{_q(h)[1]:.4f} "
          f"torch-autocast {_q(a)[0]:.4f}/{_q(a)[1]:.4f}")
    (mh, ph), (ma, pa) = _q(h), _q(a)
    assert mh >= ma - 0.01 and ph >= pa - 0.02, (mh, ma, ph, pa)


def _predictor_case(seed, S_opt, S_son, B, N, ref_device="cpu"):
    """One fitted model (seed k: data SEED_DATA + 1 + k, labels seed 3 + k, epsilons 7 + 100 k):
    the HIP f16 predictor's and torch-autocast's per-item deviations from the fp32 oracle
    (predictors.py:73-84's maths; predictive entropy as train/multimodal.py:305-306) — the
    reference's CPU path (ref_device "cpu") or the same oracle in fp32 on the GPU (TF32 off;
    7e-6 from the CPU path's entropies at 224 / 256 px, profiles/round6/pred_bisect.log)."""
    from mauv.engine import root_state
    from mauv.predict import mc_statistics
    o, m = build_pair()
    batch = make_batches(SEED_DATA + 1 + seed, 1, B=B, S_opt=S_opt, S_son=S_son)[0]
    x, b, s = batch["main_image"], batch["bathy_image"], batch["sss_image"]
    fit_model(m, *_cuda(x, b, s), torch.randint(
        0, 7, (B,), generator=torch.Generator().manual_seed(3 + seed)).cuda())
    o.load_state_dict({k: v.cpu() for k, v in m.state_dict().items()})
    bridge = EpsBridge(o, m, 7 + 100 * seed)
    if ref_device == "cpu":
        with bridge:
            pred32, var32, alea32, P32 = loops_ref.predict_batch(o, x, b, s, N)  # fp32 oracle
        bridge.collect()
        _, lg32 = oracle_replay(o, bridge.store, lambda mm: torch.stack(
            [mm(x, b, s) for _ in range(N)]).detach())
    else:
        with bridge, torch.no_grad():        # record the epsilons on a 1-triplet forward
            for _ in range(N):
                o(x[:1], b[:1], s[:1])
        bridge.collect()
        torch.backends.cudnn.allow_tf32 = False
        torch.backends.cuda.matmul.allow_tf32 = False

        def f32(mm):
            with torch.no_grad():
                lg = torch.stack([mm(*_cuda(x, b, s)) for _ in range(N)])
            P = torch.softmax(lg, -1)
            return (lg.cpu(),) + tuple(u.cpu() for u in loops_ref.mc_uncertainty_from_probs(P)) \
                + (P.cpu(),)
        _, (lg32, pred32, var32, alea32, P32) = oracle_replay(o, bridge.store, f32,
                                                              device="cuda")

    def ac(mm):
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
            lg = torch.stack([mm(*_cuda(x, b, s)) for _ in range(N)])
        P = torch.softmax(lg.float(), -1)
        return (lg.double().cpu(),) + tuple(t.cpu() for t in
                                            loops_ref.mc_uncertainty_from_probs(P)) + (P.cpu(),)
    _, (lg_ac, pred_ac, var_ac, alea_ac, P_ac) = oracle_replay(o, bridge.store, ac, device="cuda")
    root_state(m).eps_provider = bridge.provider
    with torch.no_grad(), torch.autocast("cuda"):
        st = mc_statistics(m, *_cuda(x, b, s), N, chunk=N)
    root_state(m).eps_provider = bridge.provider
    with torch.no_grad(), torch.autocast("cuda"):
        lg16 = m.mc_forward(*_cuda(x, b, s), N).double().cpu()

    def pent(P):
        pm = P.double().mean(0)
        return -(pm * torch.log(pm + 1e-8)).sum(-1)
    ref = lg32.double()
    bar = 5e-2 * ref.abs().clamp(min=1.0)
    pe32 = pent(P32)
    return dict(
        classes=len(set(pred32.tolist())),
        dl_h=(lg16 - ref).abs(), dl_a=(lg_ac - ref).abs(), ref_max=ref.abs().max().item(),
        miss_h=int(((lg16 - ref).abs() > bar).sum()), miss_a=int(((lg_ac - ref).abs() > bar).sum()),
        dv_h=(st["var"].double().cpu() - var32.double()).abs(),
        dv_a=(var_ac.double() - var32.double()).abs(),
        da_h=(st["aleatoric"].double().cpu() - alea32.double()).abs(),
        da_a=(alea_ac.double() - alea32.double()).abs(),
        dp_h=(st["predictive_entropy"].double().cpu() - pe32).abs(),
        dp_a=(pent(P_ac) - pe32).abs(),
        agree_h=(st["pred"].cpu() == pred32).float().sum().item(),
        agree_a=(pred_ac == pred32).float().sum().item(), n=B)


def _predictor_bars(rs, tag):
    cat = {k: torch.cat([r[k].flatten() for r in rs]) for k in
           ("dl_h", "dl_a", "dv_h", "dv_a", "da_h", "da_a", "dp_h", "dp_a")}
    n = sum(r["n"] for r in rs)
    agree_h, agree_a = sum(r["agree_h"] for r in rs) / n, sum(r["agree_a"] for r in rs) / n
    miss_h, miss_a = sum(r["miss_h"] for r in rs), sum(r["miss_a"] for r in rs)
    print(f"\n{tag}: {n} items, {[r['classes'] for r in rs]} classes, |logit| <= "
          f"{max(r['ref_max'] for r in rs):.1f}")
    for k, name in (("dl", "logits"), ("dv", "variance"), ("da", "aleatoric"),
                    ("dp", "pred. entropy")):
        h, a = cat[k + "_h"], cat[k + "_a"]
        print(f"  {name:13s} |d| vs fp32 oracle max/mean: HIP {h.max():.3e}/{h.mean():.3e}  "
              f"torch-autocast {a.max():.3e}/{a.mean():.3e}")
    print(f"  logits over SURVEY's 5e-2 max(1,|ref|): HIP {miss_h} torch-autocast {miss_a} of "
          f"{cat['dl_h'].numel()}; argmax agreement HIP {agree_h:.3f} autocast {agree_a:.3f}")
    assert all(r["classes"] >= 3 for r in rs)          # the class check is not degenerate
    # SURVEY §8c's 16-bit entropy bar on every item — where the reference's own scheme meets it;
    # where torch-autocast's worst item misses it too, no more than WORST_RATIO x autocast's
    for k in ("da", "dp"):
        lim = max(ENTROPY_BAR, WORST_RATIO * cat[k + "_a"].max().item())
        assert cat[k + "_h"].max() <= lim, (k, cat[k + "_h"].max().item(), lim)
    # against the reference's own scheme
    for k in ("dv", "da", "dp"):
        assert cat[k + "_h"].mean() <= MEAN_RATIO * cat[k + "_a"].mean() + 1e-7, k
    assert cat["dl_h"].mean() <= MEAN_RATIO * cat["dl_a"].mean()
    assert miss_h <= miss_a + max(2, cat["dl_h"].numel() // 500)
    assert cat["dl_h"].max() <= 5e-2 * max(1.0, max(r["ref_max"] for r in rs))
    assert agree_h >= 0.99 or agree_h >= agree_a


@pytest.mark.parametrize("S_opt,S_son,B,N", [(64, 64, 64, 32), (128, 128, 64, 32)],
                         ids=["64px", "128px"])
def test_predictor_f16_vs_torch_autocast(S_opt, S_son, B, N):
    """The drop-in predictor's default path (f16 trunks under autocast, predictors.py:55) on a
    model fitted to the batch: the module docstring's bars (ENTROPY_BAR per item, MEAN_RATIO x
    torch-autocast's mean deviations, the logit bar missed no more often than autocast).  N = 32
    MC samples (configs[3]: 100): at N = 8 (64 px, B = 64) the predictive entropy of one item
    misses SURVEY's 1e-2 in both schemes — this library 1.57e-2, torch-autocast 2.29e-2 — while
    every mean deviation of this library is at or below autocast's
    (profiles/round6/r6e_tests_B.log)."""
    _predictor_bars([_predictor_case(0, S_opt, S_son, B, N, ref_device="cuda")],
                    f"f16 predictor {S_opt}/{S_son} B={B} N={N}")


def test_predictor_f16_vs_torch_autocast_224_256_pooled():
    """The same at the configs[3] tile sizes (224 optical / 256 sonar), B=16, pooled over
    PRED_SEEDS fitted models (module docstring: one seed's mean is one draw of the rounding
    noise), with N = 32 MC samples (configs[3] draws 100: each item's entropies average the
    per-sample rounding noise over the samples as the real predictor does; at N = 8 one item of
    seed 0 sits at 1.1-1.6e-2 in BOTH schemes, profiles/round6/pred_sweep_*.log) against the
    fp32 oracle on the GPU.  Round 5 asserted this case at one seed, N = 8, with a 2.5x mean bar
    and no absolute bar."""
    _predictor_bars([_predictor_case(k, 224, 256, 16, 32, ref_device="cuda")
                     for k in range(PRED_SEEDS)],
                    f"f16 predictor 224/256 B=16 N=32, {PRED_SEEDS} seeds")
