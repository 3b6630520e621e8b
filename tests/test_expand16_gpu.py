"""The weight-stationary 16-bit expansion forwards (conv_expand16.hip): 1x1 /
stride-1 convs over K = 64 / 128 / 256 input channels into N = 256 ... 1024 outputs (the
bottleneck conv3s with the pending bn2 + ReLU on load, the layer-1 downsample without).

Against the implicit GEMM they replace (conv_pipe16, mauv_set_expand16(0)) on the same inputs:
outputs and the BN statistics partials BIT-IDENTICAL (the same MFMA chain over k, the same
rounding; one partial per 128 rows in epilogue16's canonical form: 64-row halves merged by
Chan's formula), the statistics within fp32 accumulation error (K * 2^-24 of the output scale)
of float64 statistics of the exact products (the epilogue sums the fp32 accumulators).
Ragged row counts (M % 128 in 1..127, a second half past M), several MC groups and column
groups are covered; every partial block is written (NaN-filled buffers).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"

CASES = [
    # (G, B, H, K, N, xbn)
    (2, 2, 9, 64, 256, True),       # M = 162: the last pair's second half holds 34 rows
    (1, 3, 8, 64, 256, False),      # the layer-1 downsample form (no pending BN)
    (3, 2, 10, 128, 512, True),     # M = 200: the last pair's second half is empty
    (2, 4, 16, 256, 1024, True),    # two column groups
    (1, 1, 5, 256, 1024, False),    # M = 25 < 64: one pair, one partial half
    (5, 8, 16, 128, 512, True),     # the training slice's layer-2 conv3 at B = 8
]


def _run(dt, G, B, H, K, N, xbn, expand):
    from mauv import ops
    torch.manual_seed(3)
    x = torch.randn(G, B, H, H, K, device=dev).to(dt)
    w = (torch.randn(G, N, 1, 1, K, device=dev) / K ** 0.5).to(dt)
    x_bn = (torch.rand(G, K, device=dev) + 0.5, torch.randn(G, K, device=dev) * 0.3, 1) \
        if xbn else None
    nblk = ops.fwd_stat_blocks(G, B, H, H, K, N, 1, 1, 0)
    stats = tuple(torch.full(s, float("nan"), device=dev) for s in ((G, nblk, N), (G, nblk, N),
                                                                    (G, nblk)))
    y = torch.empty(G, B, H, H, N, device=dev, dtype=dt)
    prev = ops.set_expand16(2 if expand else 0)
    try:
        ops.conv2d_fwd(x, w, y, G, B, H, H, K, N, 1, 1, 0, x_bn=x_bn, stats=stats)
    finally:
        ops.set_expand16(prev)
    torch.cuda.synchronize()
    # float64 product of the operands the kernels multiply (the pending BN: one fp32 fma, one
    # rounding to the 16-bit format, then ReLU)
    xt = x.float()
    if xbn:
        xt = torch.relu((xt * x_bn[0][:, None, None, None] + x_bn[1][:, None, None, None]).to(dt)
                        .float())
    y64 = torch.einsum("gmk,gnk->gmn", xt.double().reshape(G, -1, K),
                       w.double().reshape(G, N, K))
    return y, stats, nblk, y64


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "G{}B{}H{}K{}N{}{}".format(
    *c[:5], "x" if c[5] else ""))
def test_expand16_matches_implicit_gemm(case, dt):
    G, B, H, K, N, xbn = case
    y0, st0, nblk, _ = _run(dt, G, B, H, K, N, xbn, False)
    y1, st1, _, y64 = _run(dt, G, B, H, K, N, xbn, True)
    assert torch.equal(y0, y1)
    for t in st1:
        assert torch.isfinite(t).all()
    mean0, m20, c0 = st0
    mean1, m21, c1 = st1
    assert torch.equal(c0, c1)
    # the canonical statistics form (conv_epi16.h epilogue16 / stats_merge): bit-identical
    assert torch.equal(mean0, mean1) and torch.equal(m20, m21)
    scale = y0.float().abs().max().item() + 1e-30
    # float64 statistics of the exact products (the epilogues sum the fp32 accumulators, before
    # the 16-bit rounding of y): per 128-row block mean and M2
    M = B * H * H
    assert (y1.double().view(G, M, N) - y64).abs().max().item() <= 2 ** -7 * scale
    # fp32 accumulation over K products: |error| <= ~K * 2^-24 * max|y| per element
    tol = K * 2.0 ** -24 * scale
    for blk in range(nblk):
        rows = y64[:, 128 * blk:min(M, 128 * blk + 128)]
        mu = rows.mean(1)
        m2 = ((rows - mu[:, None]) ** 2).sum(1)
        assert (mean1[:, blk].double() - mu).abs().max().item() <= tol
        assert ((m21[:, blk].double() - m2).abs() <= 2e-5 * m2.abs() +
                2 * rows.shape[1] * tol * scale).all()
        assert (c1[:, blk] == rows.shape[1]).all()


def test_expand16_switch_round_trip():
    from mauv import ops
    prev = ops.set_expand16(False)
    assert ops.set_expand16(None) == 0
    ops.set_expand16(True)
    assert ops.set_expand16(None) == 2
    ops.set_expand16(1)
    assert ops.set_expand16(None) == 1
    ops.set_expand16(prev)
