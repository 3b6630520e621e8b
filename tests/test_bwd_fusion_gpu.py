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
