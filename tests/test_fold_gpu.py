"""A bottleneck's conv1 forming the previous block's output on load (csrc/conv_big16.hip fold,
ops.conv2d_fwd_fold) against the two passes it replaces — bn_apply (bn3 +
residual [+ the downsample branch's pending BN] + ReLU, bn.hip) and the forward conv on its
output.  The written-through block output must be BIT-identical to bn_apply's, and conv1's
output and BN-statistics partials bit-identical to the forward conv's on that output (the same
16-bit operands, the implicit GEMM's k order, epilogue16's 32-row statistic groups), within
2 ulp of a float64 reference.  Then the whole 16-bit inference forward with the fold on and off
(engine.FOLD) on the same weights and Philox samples: bit-identical logits — and a training step
(block-output ReLU bits written by the fold for the backward): bit-identical gradients.

Reference op: torchvision Bottleneck.forward's `out += identity; out = self.relu(out)` followed
by the next block's conv1 (models/base_models.py:74-90 builds the trunks)."""
import math

import pytest
import torch
import torch.nn.functional as F

from tests.golden.common import make_batches, SEED_DATA
from tests.helpers import build_pair

pytestmark = pytest.mark.gpu
dev = "cuda"
ULP = {torch.bfloat16: 2.0 ** -8, torch.float16: 2.0 ** -11}
DTYPES = [torch.bfloat16, torch.float16]


def _operands(G, B, H, W, Cin, Cout, rbn, dt):
    torch.manual_seed(29)
    y3 = torch.randn(G, B, H, W, Cin).to(dt).to(dev)
    res = torch.randn(G, B, H, W, Cin).to(dt).to(dev)
    sc = (torch.rand(G, Cin) + 0.5).to(dev)
    sh = (torch.randn(G, Cin) * 0.3).to(dev)
    res_bn = ((torch.rand(G, Cin) + 0.5).to(dev), (torch.randn(G, Cin) * 0.3).to(dev)) \
        if rbn else None
    w = (torch.randn(G, Cout, 1, 1, Cin) / math.sqrt(Cin)).to(dt).to(dev)
    return y3, sc, sh, res, res_bn, w


def _stats(ops, G, B, H, W, Cin, Cout):
    nblk = ops.fwd_stat_blocks(G, B, H, W, Cin, Cout, 1, 1, 0)
    return tuple(torch.full(s, float("nan"), device=dev) for s in
                 ((G, nblk, Cout), (G, nblk, Cout), (G, nblk)))


@pytest.mark.parametrize("dt", DTYPES, ids=["bf16", "f16"])
@pytest.mark.parametrize("G,B,H,W,Cin,Cout,rbn", [
    (2, 3, 9, 7, 256, 64, False),     # layer-1 shape, N = 64 in a 128-wide tile, ragged M
    (1, 2, 16, 16, 512, 128, True),   # a downsample block's output (pending BN on the residual)
    (2, 2, 8, 8, 1024, 256, False),   # 256-wide tiles
    (1, 2, 8, 8, 2048, 512, True),    # layer-4: 2048 channels of parameter tables in LDS
    (3, 1, 12, 12, 512, 384, False),  # ragged N (384 = 256 + 128), G = 3
])
def test_fold_bit_identical_to_bn_apply_then_conv(G, B, H, W, Cin, Cout, rbn, dt):
    from mauv import ops
    y3, sc, sh, res, res_bn, w = _operands(G, B, H, W, Cin, Cout, rbn, dt)
    M = B * H * W
    # the two passes (the training form: bn_apply_mask, whose output is bn_apply's)
    out_ref = torch.empty_like(y3)
    ops.bn_apply(y3, sc, sh, res, 1, out_ref, G, M, Cin, res_bn=res_bn)
    out_m = torch.empty_like(y3)
    mask_ref = torch.empty(y3.numel() // 8, dtype=torch.uint8, device=dev)
    ops.bn_apply_mask(y3, sc, sh, res, out_m, mask_ref, G, M, Cin, res_bn=res_bn)
    assert torch.equal(out_m, out_ref)
    y1_ref = torch.full((G, B, H, W, Cout), float("nan"), device=dev, dtype=dt)
    st_ref = _stats(ops, G, B, H, W, Cin, Cout)
    ops.conv2d_fwd(out_ref, w, y1_ref, G, B, H, W, Cin, Cout, 1, 1, 0, stats=st_ref)
    # the fold
    out = torch.full_like(y3, float("nan"))
    y1 = torch.full((G, B, H, W, Cout), float("nan"), device=dev, dtype=dt)
    st = _stats(ops, G, B, H, W, Cin, Cout)
    mask = torch.zeros(y3.numel() // 8, dtype=torch.uint8, device=dev)
    assert ops.conv2d_fwd_fold(y3, sc, sh, res, res_bn, out, w, y1, G, B, H, W, Cin, Cout,
                               stats=st, mask=mask)
    torch.cuda.synchronize()
    assert torch.equal(out, out_ref)
    assert torch.equal(mask, mask_ref)
    assert not torch.isnan(y1).any()
    assert torch.equal(y1, y1_ref)
    for a, b in zip(st, st_ref):
        assert torch.equal(a, b)
    # float64 truth on the rounded block output
    ref = torch.einsum("gmk,gnk->gmn", out_ref.double().reshape(G, M, Cin),
                       w.double().reshape(G, Cout, Cin)).reshape(G, B, H, W, Cout)
    err = (y1.double() - ref).abs().max().item()
    assert err <= 2 * ULP[dt] * ref.abs().max().item(), err
    # the block output itself against float64 bn_apply maths, rounded once
    r = res.double()
    if res_bn is not None:
        r = r * res_bn[0].double()[:, None, None, None, :] + res_bn[1].double()[:, None, None, None, :]
    ys = y3.double() * sc.double()[:, None, None, None, :]
    sh64 = sh.double()[:, None, None, None, :]
    o64 = (ys + sh64 + r).clamp_min(0)
    # one rounding to the 16-bit format (half an ulp, down to its smallest subnormal) plus the
    # fp32 fma / add roundings, which are relative to the operands (they may cancel)
    tol = ULP[dt] * o64.abs() + 2.0 ** -22 * (ys.abs() + sh64.abs() + r.abs()) + 2.0 ** -24
    assert ((out.double() - o64).abs() <= tol).all()


def test_fold_declines_uncovered_shapes_and_checks_arguments():
    from mauv import ops
    from mauv._lib import MauvError
    dt = torch.float16
    # 2112 input channels: past the kernel's 2048-channel parameter tables -> nothing launched
    G, B, H, W, Cin, Cout = 1, 1, 4, 4, 2112, 64
    y3, sc, sh, res, res_bn, w = _operands(G, B, H, W, Cin, Cout, False, dt)
    out = torch.full_like(y3, float("nan"))
    y1 = torch.full((G, B, H, W, Cout), float("nan"), device=dev, dtype=dt)
    assert not ops.conv2d_fwd_fold(y3, sc, sh, res, None, out, w, y1, G, B, H, W, Cin, Cout)
    torch.cuda.synchronize()
    assert torch.isnan(out).all() and torch.isnan(y1).all()
    # res_scale without res_shift is an argument error
    G, B, H, W, Cin, Cout = 1, 2, 8, 8, 256, 64
    y3, sc, sh, res, res_bn, w = _operands(G, B, H, W, Cin, Cout, True, dt)
    out = torch.empty_like(y3)
    y1 = torch.empty(G, B, H, W, Cout, device=dev, dtype=dt)
    with pytest.raises(MauvError):
        ops.conv2d_fwd_fold(y3, sc, sh, res, (res_bn[0], None), out, w, y1, G, B, H, W, Cin,
                            Cout)


@pytest.mark.parametrize("dt", DTYPES, ids=["bf16", "f16"])
def test_inference_forward_with_fold_is_bit_identical(dt, monkeypatch):
    from mauv import engine, ops
    from mauv.engine import root_state
    _, m = build_pair()
    engine.set_precision(m, dt)
    bt = make_batches(SEED_DATA + 5, 1, B=2, S_opt=128, S_son=128)[0]
    x, b, s = (bt[k].cuda() for k in ("main_image", "bathy_image", "sss_image"))
    ran = []
    real = ops.conv2d_fwd_fold
    monkeypatch.setattr(ops, "conv2d_fwd_fold", lambda *a, **k: ran.append(real(*a, **k)) or ran[-1])
    monkeypatch.setattr(engine, "FOLD_MIN_TILES", 0)   # fold these small launches too
    outs = []
    for fold in (False, True):
        monkeypatch.setattr(engine, "FOLD", fold)
        root_state(m).offset = 0          # the same MC samples every call
        with torch.no_grad():
            outs.append(m.mc_forward(x, b, s, 2).clone())
        torch.cuda.synchronize()
    assert not torch.isnan(outs[0]).any()
    assert torch.equal(outs[0], outs[1])
    # 3 trunks x 15 block boundaries; at 128 px the layer-4 ones (4 x 4 px, 32 rows per sample)
    # are below the kernel's 64-row minimum and run the two passes
    assert len(ran) == 45 and sum(ran) == 39, (len(ran), sum(ran))


def _train_step(m, x, b, s, y, N):
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


@pytest.mark.parametrize("dt", DTYPES, ids=["bf16", "f16"])
def test_training_step_with_fold_is_bit_identical(dt, monkeypatch):
    from mauv import engine, ops
    _, m = build_pair()
    engine.set_precision(m, dt)
    bt = make_batches(SEED_DATA + 3, 1, B=2, S_opt=64, S_son=64)[0]
    x, b, s, y = (bt[k].cuda() for k in ("main_image", "bathy_image", "sss_image", "label"))
    ran = []
    real = ops.conv2d_fwd_fold
    monkeypatch.setattr(ops, "conv2d_fwd_fold", lambda *a, **k: ran.append(real(*a, **k)) or ran[-1])
    monkeypatch.setattr(engine, "FOLD_MIN_TILES", 0)
    monkeypatch.setattr(engine, "FOLD", False)
    lg0, g0 = _train_step(m, x, b, s, y, 2)
    monkeypatch.setattr(engine, "FOLD", True)
    lg1, g1 = _train_step(m, x, b, s, y, 2)
    # 64 px: layers 1-2 (and the layer-3 entry) fold, the 4 x 4 / 2 x 2 px ones take the passes
    assert any(ran) and not all(ran), ran
    assert torch.equal(lg0, lg1)
    bad = [n for n in g0 if not torch.equal(g0[n], g1[n])]
    assert not bad, bad[:5]
