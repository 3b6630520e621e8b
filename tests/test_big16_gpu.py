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


GUARD = 4096   # sentinel elements past the end of every output buffer


def _guarded(n, dtype):
    """A buffer of n elements followed by GUARD sentinel elements (NaN), as one allocation: the
    kernels get the first n, and any write past them shows in the tail."""
    buf = torch.full((n + GUARD,), float("nan"), device=dev, dtype=dtype)
    return buf, buf[:n]


def _run(ops, x, w, G, B, H, W, Cin, Cout, R, st, pd, x_bn, big, check_tail=True):
    """big: "big16" (256-row tiles) or False (conv_pipe16).  Every output and statistics buffer
    carries a NaN tail that must survive the launch (no write past its end)."""
    prev = ops.set_big16(2 if big in (True, "big16") else 0, 512)
    try:
        Ho, Wo = ops.out_hw(H, R, st, pd), ops.out_hw(W, R, st, pd)
        nblk = ops.fwd_stat_blocks(G, B, H, W, Cin, Cout, R, st, pd)
        bufs = [_guarded(G * B * Ho * Wo * Cout, x.dtype), _guarded(G * nblk * Cout, torch.float32),
                _guarded(G * nblk * Cout, torch.float32), _guarded(G * nblk, torch.float32)]
        y = bufs[0][1].view(G, B, Ho, Wo, Cout)
        pm, pm2 = bufs[1][1].view(G, nblk, Cout), bufs[2][1].view(G, nblk, Cout)
        pc = bufs[3][1].view(G, nblk)
        ops.conv2d_fwd(x, w, y, G, B, H, W, Cin, Cout, R, st, pd, x_bn=x_bn, stats=(pm, pm2, pc))
        torch.cuda.synchronize()
        if check_tail:
            for full, body in bufs:
                assert torch.isnan(full[body.numel():].float()).all().item(), \
                    (big, "write past the end of an output buffer")
        return y, pm, pm2, pc
    finally:
        ops.set_big16(prev)


@pytest.mark.parametrize("kern", ["big16"])
@pytest.mark.parametrize("dt", DTYPES, ids=["bf16", "f16"])
@pytest.mark.parametrize("G,B,H,W,Cin,Cout,R,st,bn", [
    (2, 3, 8, 8, 512, 256, 3, 1, "relu"),     # layer-4-like 3x3, 256-wide tiles, ragged M
    (1, 2, 16, 16, 256, 256, 3, 2, "relu"),   # stride-2 3x3 (layer-3 conv2 of block 0)
    (2, 2, 9, 7, 1024, 128, 1, 1, None),      # 1x1 over 1024 channels, N = 128 tiles, odd M
    (1, 4, 8, 8, 512, 384, 1, 1, "norelu"),   # ragged N (384 = 256 + 128), BN without ReLU
    (3, 2, 6, 6, 512, 512, 1, 2, None),       # stride-2 1x1 (a downsample shape), G = 3
])
def test_big16_bit_identical_to_implicit_gemm(G, B, H, W, Cin, Cout, R, st, bn, dt, kern):
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
    yb, pmb, pm2b, pcb = _run(ops, x, w, G, B, H, W, Cin, Cout, R, st, pd, x_bn, kern)
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


@pytest.mark.parametrize("Cin,Cout,H", [(2048, 512, 64), (512, 2048, 64), (1024, 512, 256)],
                         ids=["l4c1", "l4c3", "l4.0c1"])
def test_probe_fault_shapes_through_every_forward_kernel(Cin, Cout, H):
    """The three shapes of the round-5 probe run that ended in an illegal address (G = 5,
    M = 16,384 rows per group as B = 64, H x W = H x 1 — profiles/round5/probe_fault_trace.log:
    torch.bmm's hipblasLtMatmul returned HIPBLAS_STATUS_INTERNAL_ERROR on the third and its
    fallback raised the fault; the probe's own kernels had run the first two).  Every 16-bit
    forward kernel of this library at exactly those shapes, against fp32 torch on the CPU, with a
    NaN tail behind every output buffer that must survive (an out-of-bounds write by
    a kernel launched earlier in that process would have looked the same); no vendor GEMM is
    called here.  tools/bmm_fault_probe.py runs torch.bmm alone at the third shape in a fresh
    process."""
    from mauv import ops
    G, B, W = 5, 16384 // H, 1
    g = torch.Generator().manual_seed(3)
    A = (torch.rand(G, B * H * W, Cin, generator=g) * 2 - 1).to(torch.bfloat16)
    Wt = (torch.rand(G, Cout, Cin, generator=g) * 2 - 1).to(torch.bfloat16)
    ref = torch.stack([A[i].float() @ Wt[i].float().t() for i in range(G)])
    x, w = A.to(dev), Wt.reshape(G, Cout, 1, 1, Cin).to(dev)
    for kern in (False, "big16"):
        y, _, _, _ = _run(ops, x, w, G, B, H, W, Cin, Cout, 1, 1, 0, None, kern)
        err = ((y.float().cpu().reshape(G, -1, Cout) - ref).abs().max() / ref.abs().max()).item()
        assert err <= 2 * ULP[torch.bfloat16], (kern, err)


def test_big16_switch_round_trip():
    from mauv import ops
    prev = ops.set_big16(False)
    assert prev == 1                      # default: the measured-faster shapes
    assert ops.set_big16(True) == 0
    assert ops.set_big16(prev) == 2
    assert ops.set_big16(None) == 1
