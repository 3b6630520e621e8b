"""Residual-gradient fusion of the trunk engine against its switched-off form on the same weights
and Philox epsilons (engine.py RES_MASK): a block output's residual gradient
dres = dout * relu-mask is never written — the conv1 data gradient adds dout under the block
output's mask bits and the downsample BN's backward reads dout with those bits.  dres is an
exact masking, so every gradient must be BIT-IDENTICAL to the path that stores dres (fp32 and
16-bit).
"""
import pytest
import torch

from tests.golden.common import make_batches, SEED_DATA
from tests.helpers import build_pair

pytestmark = pytest.mark.gpu


def _step(m, x, b, s, y, N):
    from mauv.engine import root_state
    from mauv.kl import get_kl_loss
    from mauv import mchead
    root_state(m).offset = 0            # the same MC samples every call
    for p in m.parameters():
        if p.grad is not None:
            p.grad.zero_()
    logits = m.mc_forward(x, b, s, N)
    ce, _, _ = mchead.mc_mean_ce(logits, y)
    (ce + get_kl_loss(m) / x.shape[0] * 0.5).backward()
    torch.cuda.synchronize()
    return logits.detach().clone(), {n: p.grad.detach().clone() for n, p in m.named_parameters()}


def _batch(B, S):
    bt = make_batches(SEED_DATA + 3, 1, B=B, S_opt=S, S_son=S)[0]
    return [bt[k].cuda() for k in ("main_image", "bathy_image", "sss_image", "label")]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16],
                         ids=["fp32", "bf16", "f16"])
def test_residual_gradient_from_mask_bits_is_exact(dt, monkeypatch):
    from mauv import engine
    _, m = build_pair()
    engine.set_precision(m, dt)
    x, b, s, y = _batch(2, 64)
    monkeypatch.setattr(engine, "RES_MASK", False)
    lg0, g0 = _step(m, x, b, s, y, 2)
    monkeypatch.setattr(engine, "RES_MASK", True)
    lg1, g1 = _step(m, x, b, s, y, 2)
    assert torch.equal(lg0, lg1)
    bad = [n for n in g0 if not torch.equal(g0[n], g1[n])]
    assert not bad, bad[:5]


@pytest.mark.parametrize("S,B", [(64, 2), (96, 3)])
def test_fp32_bn_partials_from_data_gradient_epilogue(S, B, monkeypatch):
    """engine.BWD_PARTIALS_F32: in the fp32 step the BN-backward partial sums
    of bn2 / bn1 and of the previous block's bn3 come from the LDS-staged epilogue of the data
    gradient that produces their output gradient instead of a pass over (y, dout).  The same
    fp32 terms summed in another order: logits identical; every gradient tensor within 1e-4 of
    the pass form's norm (relative L2; ADVICE r5: a cosine bar would pass a partial tile that was
    never written in a few channels — tests/test_kernels16_gpu.py fills the partials with NaN for
    that at the kernel level), the whole arena at cosine >= 0.99999."""
    from mauv import engine
    _, m = build_pair()
    x, b, s, y = _batch(B, S)
    monkeypatch.setattr(engine, "BWD_PARTIALS_F32", False)
    lg0, g0 = _step(m, x, b, s, y, 2)
    monkeypatch.setattr(engine, "BWD_PARTIALS_F32", True)
    lg1, g1 = _step(m, x, b, s, y, 2)
    assert torch.equal(lg0, lg1)
    worst, worst_rel = (1.0, None), (0.0, None)
    for n in g0:
        a, c = g0[n].double().flatten(), g1[n].double().flatten()
        if a.norm().item() == 0.0:
            assert c.norm().item() == 0.0, n
            continue
        assert torch.isfinite(c).all(), n
        cos = (a @ c).item() / (a.norm() * c.norm()).item()
        worst = min(worst, (cos, n))
        worst_rel = max(worst_rel, ((c - a).norm().item() / a.norm().item(), n))
    A = torch.cat([g0[n].double().flatten() for n in g0])
    C = torch.cat([g1[n].double().flatten() for n in g0])
    gcos = (A @ C).item() / (A.norm() * C.norm()).item()
    print(f"fp32 {S} px B={B}: whole arena cosine {gcos:.9f}, worst tensor cosine {worst}, "
          f"worst relative L2 difference {worst_rel}")
    assert gcos >= 0.99999 and worst_rel[0] <= 1e-4, (gcos, worst, worst_rel)
