"""The 16-bit 3x3 / stride-1 / 64 -> 64 forward through an LDS image of the input rows
(csrc/conv_halo16.hip) against the implicit GEMM it replaces (conv_pipe16.hip, selected with
ops.set_halo3(False)): the same operands (the pending BN applied on load, rounded once), the
same accumulation order, so outputs and BN statistics partials must be BIT-identical — and
both within 2 ulp of a float64 reference.  Shapes cover both tile heights (256 pixels when the
tile spans whole rows, else 128), tiles that cross image boundaries in the flattened row space,
ragged last tiles, non-square images and one-row images."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"
DTYPES = [torch.bfloat16, torch.float16]
ULP = {torch.bfloat16: 2.0 ** -8, torch.float16: 2.0 ** -11}


def _run(ops, x, w, G, B, H, W, x_bn, halo):
    prev = ops.set_halo3(halo)
    try:
        y = torch.empty(G, B, H, W, 64, device=dev, dtype=x.dtype)
        nblk = ops.fwd_stat_blocks(G, B, H, W, 64, 64, 3, 1, 1)
        pm = torch.full((G, nblk, 64), float("nan"), device=dev)
        pm2 = torch.full((G, nblk, 64), float("nan"), device=dev)
        pc = torch.full((G, nblk), float("nan"), device=dev)
        ops.conv2d_fwd(x, w, y, G, B, H, W, 64, 64, 3, 1, 1, x_bn=x_bn, stats=(pm, pm2, pc))
        torch.cuda.synchronize()
        return y, pm, pm2, pc
    finally:
        ops.set_halo3(prev)


@pytest.mark.parametrize("dt", DTYPES, ids=["bf16", "f16"])
@pytest.mark.parametrize("G,B,H,W,bn", [
    (2, 3, 16, 16, "relu"),    # 256-pixel tiles (one image per tile), pending BN + ReLU
    (1, 2, 14, 56, "relu"),    # W = 56: 128-pixel tiles crossing rows and images
    (2, 2, 9, 56, None),       # ragged last tile, no pending BN
    (1, 3, 7, 12, "norelu"),   # 256-pixel tiles spanning several images; BN without ReLU
    (3, 2, 5, 8, "relu"),      # W = 8: 32 rows per tile, many image boundaries
    (1, 2, 1, 64, "relu"),     # one-row images: every vertical tap is padding
    (2, 2, 12, 64, "relu"),    # W = 64 (the bench's bathymetry / SSS trunks), 4 rows per tile
])
def test_halo3_bit_identical_to_implicit_gemm(G, B, H, W, bn, dt):
    from mauv import ops
    torch.manual_seed(11)
    x = torch.randn(G, B, H, W, 64).to(dt).to(dev)
    w = (torch.randn(G, 64, 3, 3, 64) / math.sqrt(64 * 9)).to(dt).to(dev)
    x_bn = None
    if bn is not None:
        sc = (torch.rand(G, 64) + 0.5).to(dev)
        sh = (torch.randn(G, 64) * 0.2).to(dev)
        x_bn = (sc, sh, 1 if bn == "relu" else 0)
    yh, pmh, pm2h, pch = _run(ops, x, w, G, B, H, W, x_bn, True)
    yg, pmg, pm2g, pcg = _run(ops, x, w, G, B, H, W, x_bn, False)
    assert torch.equal(yh, yg)
    assert torch.equal(pmh, pmg) and torch.equal(pm2h, pm2g) and torch.equal(pch, pcg)
    # float64 truth on the same rounded operands
    xin = x.double()
    if x_bn is not None:
        xin = xin * sc.double()[:, None, None, None, :] + sh.double()[:, None, None, None, :]
        if bn == "relu":
            xin = xin.clamp_min(0)
        xin = xin.to(dt).double()       # the loader rounds the normalised input once
    ref = torch.stack([F.conv2d(xin[g].permute(0, 3, 1, 2), w[g].double().permute(0, 3, 1, 2),
                                padding=1).permute(0, 2, 3, 1) for g in range(G)])
    err = (yh.double() - ref).abs().max().item()
    assert err <= 2 * ULP[dt] * ref.abs().max().item(), err
    # the statistics partials describe y's fp32 pre-rounding values: counts sum to the rows
    assert torch.equal(pch.sum(1), torch.full((G,), float(B * H * W), device=dev))
    mean = (pmh * pch[..., None]).sum(1) / pch.sum(1)[:, None]
    assert torch.allclose(mean.double(), ref.mean((1, 2, 3)), rtol=1e-3, atol=1e-4)


def test_halo3_switch_round_trip():
    from mauv import ops
    prev = ops.set_halo3(False)
    assert ops.set_halo3(True) is False
    assert ops.set_halo3(prev) is True


@pytest.mark.parametrize("dt", DTYPES, ids=["bf16", "f16"])
@pytest.mark.parametrize("G,B,H,W,mode", [
    (2, 3, 16, 16, "addend"),   # 256-pixel tiles, the residual addend (identity block's conv1 role)
    (1, 2, 14, 56, "plain"),    # W = 56: 128-pixel tiles crossing rows and images
    (2, 2, 9, 56, "accumulate"),  # ragged last tile, accumulate into dx
    (3, 2, 5, 8, "mask"),       # the addend under ReLU-mask bits, many image boundaries
    (1, 2, 1, 64, "plain"),     # one-row images
    (2, 2, 12, 64, "addend"),   # W = 64 (bathymetry / SSS trunks)
])
def test_halo3_dgrad_bit_identical_to_implicit_gemm(G, B, H, W, mode, dt):
    """The 3x3 / stride-1 64 -> 64 data gradient through the LDS row image (taps mirrored, the
    weights as a column image) equals the implicit GEMM bit for bit, epilogue forms included."""
    from mauv import ops
    torch.manual_seed(12)
    dy = torch.randn(G, B, H, W, 64).to(dt).to(dev)
    w = (torch.randn(G, 64, 3, 3, 64) / math.sqrt(64 * 9)).to(dt).to(dev)
    addend = torch.randn(G, B, H, W, 64).to(dt).to(dev) if mode in ("addend", "mask") else None
    mask = None
    if mode == "mask":
        mask = torch.randint(0, 256, (G * B * H * W * 64 // 8,), dtype=torch.uint8, device=dev)
    base = torch.randn(G, B, H, W, 64).to(dt).to(dev)
    outs = []
    for halo in (True, False):
        prev = ops.set_halo3(halo)
        try:
            dx = base.clone() if mode == "accumulate" else torch.empty_like(base)
            ops.conv2d_bwd_data(dy, w, dx, G, B, H, W, 64, 64, 3, 1, 1, addend=addend,
                                accumulate=mode == "accumulate", addend_mask=mask)
            torch.cuda.synchronize()
            outs.append(dx)
        finally:
            ops.set_halo3(prev)
    assert torch.equal(outs[0], outs[1])
    ref = torch.stack([F.conv_transpose2d(dy[g].double().permute(0, 3, 1, 2),
                                          w[g].double().permute(0, 3, 1, 2), padding=1)
                       .permute(0, 2, 3, 1) for g in range(G)])
    if mode == "accumulate":
        ref = ref + base.double()
    elif mode == "addend":
        ref = ref + addend.double()
    elif mode == "mask":
        bits = ((mask[:, None].int() >> torch.arange(8, device=dev)) & 1).reshape(ref.shape)
        ref = ref + addend.double() * bits
    err = (outs[0].double() - ref).abs().max().item()
    assert err <= 4 * ULP[dt] * ref.abs().max().item(), err
