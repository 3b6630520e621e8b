"""The 16-bit forward on 256-row tiles with LDS-DMA operands (csrc/conv_big16.hip) against the
implicit GEMM it replaces for long-K forwards (conv_pipe16.hip, selected with
ops.set_big16(False)): the same operands (the pending BN applied to the landed tile, rounded
once, zero outside the image) and the same k order per output element, and the statistics
epilogue adds the same 32-row groups in the same order, so outputs and BN statistics partials
must be BIT-identical — and within 2 ulp of a float64 reference.  Shapes: 1x1 and 3x3, stride 1 and 2, N = 128
and 256-wide tiles, ragged M, pending BN with and without ReLU, several MC groups."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"
DTYPES = [torch.bfloat16, torch.float16]
ULP = {torch.bfloat16: 2.0 ** -8, torch.float16: 2.0 ** -11}


def _run(ops, x, w, G, B, H, W, Cin, Cout, R, st, pd, x_bn, big):
    prev = ops.set_big16(2 if big else 0, 512)
    try:
        Ho, Wo = ops.out_hw(H, R, st, pd), ops.out_hw(W, R, st, pd)
        y = torch.full((G, B, Ho, Wo, Cout), float("nan"), device=dev, dtype=x.dtype)
        nblk = ops.fwd_stat_blocks(G, B, H, W, Cin, Cout, R, st, pd)
        pm = torch.full((G, nblk, Cout), float("nan"), device=dev)
        pm2 = torch.full((G, nblk, Cout), float("nan"), device=dev)
        pc = torch.full((G, nblk), float("nan"), device=dev)
        ops.conv2d_fwd(x, w, y, G, B, H, W, Cin, Cout, R, st, pd, x_bn=x_bn, stats=(pm, pm2, pc))
        torch.cuda.synchronize()
        return y, pm, pm2, pc
    finally:
        ops.set_big16(prev)


@pytest.mark.parametrize("dt", DTYPES, ids=["bf16", "f16"])
@pytest.mark.parametrize("G,B,H,W,Cin,Cout,R,st,bn", [
    (2, 3, 8, 8, 512, 256, 3, 1, "relu"),     # layer-4-like 3x3, 256-wide tiles, ragged M
    (1, 2, 16, 16, 256, 256, 3, 2, "relu"),   # stride-2 3x3 (layer-3 conv2 of block 0)
    (2, 2, 9, 7, 1024, 128, 1, 1, None),      # 1x1 over 1024 channels, N = 128 tiles, odd M
    (1, 4, 8, 8, 512, 384, 1, 1, "norelu"),   # ragged N (384 = 256 + 128), BN without ReLU
    (3, 2, 6, 6, 512, 512, 1, 2, None),       # stride-2 1x1 (a downsample shape), G = 3
])
def test_big16_bit_identical_to_implicit_gemm(G, B, H, W, Cin, Cout, R, st, bn, dt):
    from mauv import ops
    torch.manual_seed(13)
    pd = R // 2
    x = torch.randn(G, B, H, W, Cin).to(dt).to(dev)
    w = (torch.randn(G, Cout, R, R, Cin) / math.sqrt(Cin * R * R)).to(dt).to(dev)
    x_bn = None
    if bn is not None:
        sc = (torch.rand(G, Cin) + 0.5).to(dev)
        sh = (torch.randn(G, Cin) * 0.2).to(dev)
        x_bn = (sc, sh, 1 if bn == "relu" else 0)
    yb, pmb, pm2b, pcb = _run(ops, x, w, G, B, H, W, Cin, Cout, R, st, pd, x_bn, True)
    yg, pmg, pm2g, pcg = _run(ops, x, w, G, B, H, W, Cin, Cout, R, st, pd, x_bn, False)
    assert not torch.isnan(yb).any()
    assert torch.equal(yb, yg)
    # the statistics partials sum the same 32-row groups in the same order (epilogue16)
    assert torch.equal(pcb, pcg) and torch.equal(pmb, pmg) and torch.equal(pm2b, pm2g)
    # float64 truth on the same rounded operands
    xin = x.double()
    if x_bn is not None:
        xin = xin * sc.double()[:, None, None, None, :] + sh.double()[:, None, None, None, :]
        if bn == "relu":
            xin = xin.clamp_min(0)
        xin = xin.to(dt).double()       # the transform rounds the normalised input once
    ref = torch.stack([F.conv2d(xin[g].permute(0, 3, 1, 2), w[g].double().permute(0, 3, 1, 2),
                                stride=st, padding=pd).permute(0, 2, 3, 1) for g in range(G)])
    err = (yb.double() - ref).abs().max().item()
    assert err <= 2 * ULP[dt] * ref.abs().max().item(), err


def test_big16_switch_round_trip():
    from mauv import ops
    prev = ops.set_big16(False)
    assert prev == 1                      # default: the measured-faster shapes
    assert ops.set_big16(True) == 0
    assert ops.set_big16(prev) == 2
    assert ops.set_big16(None) == 1
