"""The 16-bit 3x3 forwards over 128-512 channels through the chunked LDS row image
(conv_haloc16.hip): the layer-2..4 bottleneck conv2s, the pending bn1 + ReLU
applied on load; both wave-tile forms (32 x 64, the default, and 64 x 64).

Against float64 convolutions of the exact operands the kernels multiply, and against the
implicit GEMM the kernel replaces (conv_pipe16, mauv_set_haloc16(0)) on the same inputs.  The two
kernels sum the 9 * Cin products in different orders ((chunk, tap, k) here, (tap, chunk, k)
there), so outputs agree to fp32 summation error before the 16-bit rounding: within one 16-bit
rounding step of the output scale of each other and of float64.  The statistics partials (one
per 128 rows, epilogue16's canonical form) within fp32 accumulation error (9 * Cin * 2^-24 of the
output scale) of float64 statistics.  Ragged row counts, widths that do not divide 128 (a tile
spanning partial rows), image boundaries inside a tile, several MC groups and column tiles are
covered; every partial block is written (NaN-filled buffers).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"

CASES = [
    # (G, B, H, W, C, N, xbn)
    (2, 2, 8, 8, 128, 128, True),       # layer-2 form, tiles aligned to whole images
    (1, 3, 10, 12, 128, 256, True),     # W = 12: tiles span partial rows; M = 360 ragged
    (2, 2, 16, 16, 256, 256, False),    # no pending BN
    (1, 2, 7, 7, 512, 512, True),       # layer-4 form at 7 x 7: four column tiles, M = 98
    (3, 1, 32, 32, 128, 128, True),     # W = 32: four rows per tile
    (1, 5, 4, 4, 256, 128, True),       # W = 4: 32 rows per tile, 8 images in one tile
    (2, 2, 8, 8, 128, 128, "norelu"),   # a pending BN without the ReLU
]


def _run(dt, G, B, H, W, C, N, xbn, haloc):
    from mauv import ops
    torch.manual_seed(5)
    x = torch.randn(G, B, H, W, C, device=dev).to(dt)
    w = (torch.randn(G, N, 3, 3, C, device=dev) / (9 * C) ** 0.5).to(dt)
    relu = xbn != "norelu"
    x_bn = (torch.rand(G, C, device=dev) + 0.5, torch.randn(G, C, device=dev) * 0.3, int(relu)) \
        if xbn else None
    nblk = ops.fwd_stat_blocks(G, B, H, W, C, N, 3, 1, 1)
    stats = tuple(torch.full(s, float("nan"), device=dev) for s in ((G, nblk, N), (G, nblk, N),
                                                                    (G, nblk)))
    y = torch.empty(G, B, H, W, N, device=dev, dtype=dt)
    prev = ops.set_haloc16(haloc)
    try:
        ops.conv2d_fwd(x, w, y, G, B, H, W, C, N, 3, 1, 1, x_bn=x_bn, stats=stats)
    finally:
        ops.set_haloc16(prev)
    torch.cuda.synchronize()
    # float64 convolution of the operands the kernels multiply (the pending BN: one fp32 fma,
    # one rounding to the 16-bit format, then ReLU)
    xt = x.float()
    if xbn:
        xt = (xt * x_bn[0][:, None, None, None] + x_bn[1][:, None, None, None]).to(dt).float()
        if relu:
            xt = torch.relu(xt)
    y64 = torch.stack([
        F.conv2d(xt[g].double().permute(0, 3, 1, 2), w[g].double().permute(0, 3, 1, 2), padding=1)
        .permute(0, 2, 3, 1) for g in range(G)]).reshape(G, B * H * W, N)
    return y, stats, nblk, y64


@pytest.mark.parametrize("mode", [1, 2], ids=["w32x64", "w64x64"])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "G{}B{}H{}W{}C{}N{}{}".format(
    *c[:6], {True: "x", False: "", "norelu": "xn"}[c[6]]))
def test_haloc16_matches_float64_and_implicit_gemm(case, dt, mode):
    G, B, H, W, C, N, xbn = case
    y0, st0, nblk, _ = _run(dt, G, B, H, W, C, N, xbn, 0)
    y1, st1, _, y64 = _run(dt, G, B, H, W, C, N, xbn, mode)
    M = B * H * W
    for t in st1:
        assert torch.isfinite(t).all()
    scale = y64.abs().max().item() + 1e-30
    ulp = 2.0 ** (-8 if dt == torch.bfloat16 else -11)  # half a 16-bit step of a value in [1, 2)
    # one 16-bit rounding step of the output scale (+ fp32 summation error, far below it)
    bound = 2 * ulp * scale
    assert (y1.double().view(G, M, N) - y64).abs().max().item() <= bound
    assert (y1.double() - y0.double()).abs().max().item() <= 2 * bound
    mean1, m21, c1 = st1
    assert torch.equal(c1, st0[2])
    tol = 9 * C * 2.0 ** -24 * scale
    for blk in range(nblk):
        rows = y64[:, 128 * blk:min(M, 128 * blk + 128)]
        mu = rows.mean(1)
        m2 = ((rows - mu[:, None]) ** 2).sum(1)
        assert (mean1[:, blk].double() - mu).abs().max().item() <= tol
        assert ((m21[:, blk].double() - m2).abs() <= 2e-5 * m2.abs() +
                2 * rows.shape[1] * tol * scale).all()
        assert (c1[:, blk] == rows.shape[1]).all()


def test_haloc16_switch_round_trip():
    from mauv import ops
    prev = ops.set_haloc16(False)
    assert ops.set_haloc16(None) == 0
    ops.set_haloc16(True)
    assert ops.set_haloc16(None) == 1
    ops.set_haloc16(2)
    assert ops.set_haloc16(None) == 2
    ops.set_haloc16(3)
    assert ops.set_haloc16(None) == 3
    ops.set_haloc16(prev)


DGRAD_CASES = [
    # (G, B, H, W, C (= Cin = Cout), form)
    (2, 2, 8, 8, 128, "plain"),
    (1, 3, 10, 12, 256, "addend"),       # tiles spanning partial rows, M = 360 ragged
    (2, 2, 7, 7, 512, "accumulate"),
    (3, 1, 16, 16, 128, "mask"),         # addend counted under ReLU-mask bits
]


@pytest.mark.parametrize("mode", [1, 2], ids=["w32x64", "w64x64"])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("case", DGRAD_CASES, ids=lambda c: "G{}B{}H{}W{}C{}-{}".format(*c))
def test_haloc16_dgrad_matches_float64_and_implicit_gemm(case, dt, mode):
    """The 3x3 / stride-1 data gradients over 128-512 channels (mode 1 / 2) against the
    implicit GEMM (mode 3: forwards only) and, plain, against float64: dx within one 16-bit
    rounding step of the output scale; the addend / accumulate / mask forms through the same
    epilogue."""
    from mauv import ops
    G, B, H, W, C, form = case
    torch.manual_seed(7)
    dy = torch.randn(G, B, H, W, C, device=dev).to(dt)
    w = (torch.randn(G, C, 3, 3, C, device=dev) / (9 * C) ** 0.5).to(dt)
    add = torch.randn(G, B, H, W, C, device=dev).to(dt) if form in ("addend", "mask") else None
    mask = (torch.randint(0, 256, (G * B * H * W * C // 8,), device=dev, dtype=torch.uint8)
            if form == "mask" else None)
    base = torch.randn(G, B, H, W, C, device=dev).to(dt) if form == "accumulate" else None
    outs = []
    for m in (3, mode):
        dx = base.clone() if base is not None else torch.empty(G, B, H, W, C, device=dev,
                                                                dtype=dt)
        prev = ops.set_haloc16(m)
        try:
            ops.conv2d_bwd_data(dy, w, dx, G, B, H, W, C, C, 3, 1, 1, addend=add,
                                accumulate=form == "accumulate", addend_mask=mask)
        finally:
            ops.set_haloc16(prev)
        torch.cuda.synchronize()
        outs.append(dx.double())
    ulp = 2.0 ** (-8 if dt == torch.bfloat16 else -11)
    scale = outs[0].abs().max().item() + 1e-30
    assert torch.isfinite(outs[1]).all()
    assert (outs[1] - outs[0]).abs().max().item() <= 4 * ulp * scale
    if form == "plain":
        ref = torch.stack([
            F.conv_transpose2d(dy[g].double().permute(0, 3, 1, 2),
                               w[g].double().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
            for g in range(G)])
        assert (outs[1] - ref).abs().max().item() <= 2 * ulp * (ref.abs().max().item() + 1e-30)
