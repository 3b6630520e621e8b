"""16-bit HIP paths judged against the reference's OWN mixed-precision scheme.

The bar: the oracle run under ``torch.autocast("cuda", dtype)`` on
the same GPU, with the same weights and epsilons — what ``inference/predictors.py:55`` does on
CUDA, and what a bf16 autocast training step of the reference would compute.  The HIP path
must be at least as close to the truth (float64 oracle for gradients, fp32 oracle for the
predictor's statistics) as that scheme, within a stated margin.

* bf16 training step at the BASELINE tile sizes (224 optical / 256 sonar), B=4, N=2: the
  cosine of EVERY parameter tensor's gradient (trunks included) with the float64 truth is no
  worse than torch-autocast's cosine for that tensor by more than ``COS_MARGIN``, and the
  median over tensors is no worse than autocast's median.
* f16 predictor (the drop-in default path, ``multimodal_predict_and_save``'s maths) at B=64,
  N=8: predictive variance and aleatoric uncertainty deviate from the fp32 oracle by at most
  2x what torch-autocast deviates (max over items), and the predicted class agrees with the
  fp32 oracle on >= 99 % of the items over a head whose argmax depends on the
  input (``spread_head``: at random init every item would otherwise be class 4).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import bayes_ref, loops_ref
from tests.golden.common import make_batches, SEED_DATA
from tests.helpers import build_pair, EpsBridge, oracle_replay, cosines, spread_head

pytestmark = pytest.mark.gpu

COS_MARGIN = 0.02    # per tensor: cos(HIP) >= cos(autocast) - COS_MARGIN


def _cuda(*ts):
    return [t.cuda() for t in ts]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("S_opt,S_son,B,N", [(224, 256, 4, 2), (64, 64, 2, 3)],
                         ids=["224-256", "64"])
def test_train_step16_grads_vs_torch_autocast(dt, S_opt, S_son, B, N):
    from mauv.engine import root_state, set_precision
    from mauv.kl import get_kl_loss
    from mauv import mchead
    o, m = build_pair()
    set_precision(m, dt)
    batch = make_batches(SEED_DATA, 1, B=B, S_opt=S_opt, S_son=S_son)[0]
    x, b, s, y = batch["main_image"], batch["bathy_image"], batch["sss_image"], batch["label"]

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

    bridge = EpsBridge(o, m, 99)
    with bridge, torch.no_grad():          # records the epsilons (fp32 CPU forward)
        for _ in range(N):
            o(x, b, s)
    bridge.collect()
    o64, (lg64, _) = oracle_replay(o, bridge.store, lambda mm: loss_of(mm, "cpu", torch.float64),
                                   dtype=torch.float64)
    oac, (lgac, _) = oracle_replay(o, bridge.store, lambda mm: loss_of(mm, "cuda", amp=dt),
                                   device="cuda")
    root_state(m).eps_provider = bridge.provider
    logits = m.mc_forward(*_cuda(x, b, s), N)
    ce, _, _ = mchead.mc_mean_ce(logits, y.cuda())
    (ce + get_kl_loss(m) / B * 0.5).backward()

    truth = list(o64.parameters())
    c_hip = cosines(list(m.named_parameters()), truth)
    c_ac = cosines(list(oac.named_parameters()), truth)
    assert set(c_hip) == set(c_ac) and len(c_hip) > 600, len(c_hip)
    names = sorted(c_hip)
    h = np.array([c_hip[n] for n in names])
    a = np.array([c_ac[n] for n in names])
    trunk = np.array([n.split(".")[0].endswith("_feat") for n in names])
    print(f"\n{dt} {S_opt}/{S_son} B={B} N={N}: {len(names)} tensors ({trunk.sum()} trunk); "
          f"cos vs fp64 median/p10/min  HIP {np.median(h):.5f}/{np.quantile(h, .1):.5f}/"
          f"{h.min():.5f}  torch-autocast {np.median(a):.5f}/{np.quantile(a, .1):.5f}/"
          f"{a.min():.5f}; worst HIP-autocast {np.min(h - a):+.5f} "
          f"({names[int(np.argmin(h - a))]})")
    for n, hv, av in zip(names, h, a):
        assert hv >= av - COS_MARGIN, (n, hv, av)
    assert np.median(h) >= np.median(a) - 1e-3
    # logits: both schemes against the float64 truth
    dh = (logits.detach().double().cpu() - lg64.detach()).abs().max().item()
    da = (lgac.detach().double().cpu() - lg64.detach()).abs().max().item()
    print(f"max |dlogit| vs fp64: HIP {dh:.3e}  torch-autocast {da:.3e}")
    assert dh <= max(2 * da, 1e-3)


@pytest.mark.parametrize("S", [64, 128], ids=["64px", "128px"])
def test_predictor_f16_vs_torch_autocast(S):
    """The drop-in predictor's default path (f16 trunks under autocast, predictors.py:55)."""
    from mauv.engine import root_state
    from mauv.predict import mc_statistics
    o, m = build_pair()
    spread_head(o, m)
    B, N = 64, 8
    batch = make_batches(SEED_DATA + 1, 1, B=B, S_opt=S, S_son=S)[0]
    x, b, s = batch["main_image"], batch["bathy_image"], batch["sss_image"]
    bridge = EpsBridge(o, m, 7)
    with bridge:
        pred32, var32, alea32, _ = loops_ref.predict_batch(o, x, b, s, N)   # fp32 oracle
    bridge.collect()

    def ac(mm):
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
            return loops_ref.predict_batch(mm, *_cuda(x, b, s), N)
    _, (pred_ac, var_ac, alea_ac, _) = oracle_replay(o, bridge.store, ac, device="cuda")
    root_state(m).eps_provider = bridge.provider
    with torch.no_grad(), torch.autocast("cuda"):
        st = mc_statistics(m, *_cuda(x, b, s), N, chunk=N)
    classes = len(set(pred32.tolist()))
    dv_h = (st["var"].double().cpu() - var32.double()).abs().max().item()
    dv_a = (var_ac.double().cpu() - var32.double()).abs().max().item()
    da_h = (st["aleatoric"].double().cpu() - alea32.double()).abs().max().item()
    da_a = (alea_ac.double().cpu() - alea32.double()).abs().max().item()
    agree = (st["pred"].cpu() == pred32).float().mean().item()
    agree_ac = (pred_ac.cpu() == pred32).float().mean().item()
    print(f"\nS={S} B={B} N={N}: {classes} classes predicted; |dvar| HIP {dv_h:.3e} autocast "
          f"{dv_a:.3e}; |dalea| HIP {da_h:.3e} autocast {da_a:.3e}; argmax agreement HIP "
          f"{agree:.3f} autocast {agree_ac:.3f}")
    assert classes >= 3            # the class check is not degenerate
    assert dv_h <= 2 * dv_a + 1e-7
    assert da_h <= 2 * da_a + 1e-6
    assert agree >= 0.99
