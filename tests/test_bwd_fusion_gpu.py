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


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
def test_bn_partials_from_data_gradient_epilogue(dt, monkeypatch):
    """engine.BWD_PARTIALS: bn1 / bn2's backward partial sums come from the
    epilogue of the data gradient that produces their output gradient instead of a pass over
    (y, dout).  The sums are the same terms in another fp32 order, so gradients are not
    bit-identical; the 16-bit backward amplifies the last-bit differences along the chain (the
    stem's BN parameters, summed over every pixel, see them most).  Bar: logits identical, the
    whole gradient arena at cosine >= ARENA[dt], every tensor at cosine >= COS[dt] (measured:
    bf16 0.99989 / worst tensor 0.9956, the image stem's bn1.bias; f16 0.99997 / 0.99990)."""
    from mauv import engine
    COS = {torch.bfloat16: 0.99, torch.float16: 0.999}
    ARENA = {torch.bfloat16: 0.9995, torch.float16: 0.9999}
    _, m = build_pair()
    engine.set_precision(m, dt)
    x, b, s, y = _batch(2, 64)
    monkeypatch.setattr(engine, "BWD_PARTIALS", False)
    lg0, g0 = _step(m, x, b, s, y, 2)
    monkeypatch.setattr(engine, "BWD_PARTIALS", True)
    lg1, g1 = _step(m, x, b, s, y, 2)
    assert torch.equal(lg0, lg1)
    rows = []
    for n in g0:
        a, c = g0[n].double().flatten(), g1[n].double().flatten()
        na = a.norm().item()
        if na == 0.0:
            assert c.norm().item() == 0.0, n
            continue
        cos = (a @ c).item() / (na * c.norm().item() + 1e-300)
        rows.append((cos, (a - c).norm().item() / na, n))
    rows.sort()
    for cos, rel, n in rows[:5]:
        print(f"{dt} {n}: cosine {cos:.6f}, relative L2 {rel:.2e}")
    A = torch.cat([g0[n].double().flatten() for n in g0])
    C = torch.cat([g1[n].double().flatten() for n in g0])
    gcos = (A @ C).item() / (A.norm() * C.norm()).item()
    print(f"{dt} whole arena: cosine {gcos:.8f}")
    assert gcos >= ARENA[dt]
    assert rows[0][0] >= COS[dt], rows[:3]
