"""Centred 16-bit storage of the BatchNorm inputs (ConvArgs::ysh, ops.conv2d_fwd(ysh=...),
engine.CENTRE_Y) on every 16-bit forward route and in the statistics finalize.

A conv output that feeds a batch-statistics BatchNorm is stored as round16(y - c), c = that BN's
centre: every 16-bit forward kernel starts its fp32 accumulators at -c (conv_epi16.h
acc_start16), so the stored values and the statistics partials are those of y - c.  Checked here:
* every forward kernel (the implicit GEMM's one-stage, short-K and long-K forms, the 3x3 LDS row
  images over 64 and 128 channels, the 256-row LDS-DMA tiles, the weight-stationary expansions,
  the stems over shared im2col rows, the fold): the stored values within 2 ulp of float64
  (conv - c); the partial means those of the uncentred run minus c and the M2 partials equal,
  to fp32 rounding; — inputs with a large channel mean, c near it — the reconstructed
  y = stored + c closer to float64 than the uncentred store, in BatchNorm's units (the point of
  the change); and every route that keeps the implicit GEMM's k order (all but the chunked
  3x3 row image) BIT-identical to it with the same centre, outputs and statistics;
* mauv_bn_stats_finalize with y_shift on the centred partials: scale that of the uncentred
  finalize (to fp32 rounding of the merge), mean = the stored values' mean, shift such that stored * scale + shift =
  y * scale + shift_uncentred, the running statistics those of the true mean, and y_shift
  aliasing run_mean gives the same result as a copy of it (it is read before the update).
Reference op: F.conv2d followed by F.batch_norm in training mode inside torchvision's
Bottleneck / stem (models/base_models.py:74-90)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"
DTYPES = [torch.bfloat16, torch.float16]
ULP = {torch.bfloat16: 2.0 ** -8, torch.float16: 2.0 ** -11}

# (route, G, B, H, Cin, Cout, R, stride, pad): the route forced through MauvRoute
ROUTES = [
    ("pipe16", 2, 2, 9, 64, 256, 1, 1, 0),      # one-stage K = 64
    ("pipe16", 2, 3, 9, 128, 256, 1, 1, 0),     # short-K sequential K = 128
    ("pipe16", 1, 2, 8, 256, 512, 1, 2, 0),     # strided 1x1 (a downsample)
    ("pipe16", 2, 2, 12, 64, 128, 3, 2, 1),     # long-K 3x3 stride 2
    ("halo3", 2, 2, 10, 64, 64, 3, 1, 1),       # 3x3 64 -> 64 row image
    ("haloc16", 2, 2, 8, 128, 128, 3, 1, 1),    # 3x3 128 -> 128 chunked row image
    ("big16", 2, 2, 16, 512, 256, 1, 1, 0),     # 256-row LDS-DMA tiles
    ("expand16", 2, 4, 16, 128, 512, 1, 1, 0),  # weight-stationary K = 128
    ("expand16", 2, 4, 16, 256, 1024, 1, 1, 0),  # weight-stationary K = 256
]
ROUTE_SET = {
    "pipe16": dict(big16=0, expand16=0, haloc16=0, halo3=0),
    "halo3": dict(big16=0, expand16=0, haloc16=0, halo3=1),
    "haloc16": dict(big16=0, expand16=0, haloc16=1, halo3=0),
    "big16": dict(big16=2, big16_min_k=512, expand16=0, haloc16=0, halo3=0),
    "expand16": dict(big16=0, expand16=2, haloc16=0, halo3=0),
}


def _stat_bufs(ops, G, B, H, Cin, Cout, R, st, pd):
    nblk = ops.fwd_stat_blocks(G, B, H, H, Cin, Cout, R, st, pd)
    return tuple(torch.full(s, float("nan"), device=dev) for s in
                 ((G, nblk, Cout), (G, nblk, Cout), (G, nblk)))


def _large_mean_operands(G, B, H, Cin, Cout, R, dt, seed=7):
    """Non-negative inputs (post-ReLU activations) and weights with a per-output-channel bias in
    their sum, so every output channel has a mean several times its spread — where an uncentred
    16-bit store loses the most against BatchNorm's 1/std."""
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(G, B, H, H, Cin, generator=g).to(dt)
    w = torch.randn(G, Cout, R, R, Cin, generator=g) / math.sqrt(Cin * R * R)
    w = w + (torch.rand(1, Cout, 1, 1, 1, generator=g) * 8 - 4) / (Cin * R * R)
    return x, w.to(dt)


def _ref(x, w, st, pd):
    return torch.stack([F.conv2d(x[g].permute(0, 3, 1, 2).double(),
                                 w[g].permute(0, 3, 1, 2).double(), stride=st,
                                 padding=pd).permute(0, 2, 3, 1) for g in range(w.shape[0])])


def _check_stats(s0, s1, c):
    """Statistics partials of the centred run (s1) against the uncentred run's (s0): counts
    equal, means shifted by the centre, M2 equal — to fp32 rounding of the accumulations."""
    (m0, q0, n0), (m1, q1, n1) = s0, s1
    assert torch.equal(n0, n1)
    cc = c.view(1, 1, -1)
    assert torch.allclose(m1, m0 - cc, rtol=0, atol=1e-5 * max(1.0, m0.abs().max().item()))
    assert torch.allclose(q1, q0, rtol=1e-4, atol=1e-4 * q0.abs().max().item())


def _check_centred(y0, y1, c, ref, dt, tag):
    """y0 uncentred, y1 centred (stored y - c) against the float64 truth ref.  The error that
    matters is the one BatchNorm sees, relative to each channel's spread: the rms error of
    y = stored + c over a channel divided by that channel's standard deviation, averaged over
    the channels — the centred store must at least halve it on these large-mean operands."""
    c64 = c.double().cpu()
    ref = ref.cpu()
    e1 = (y1.double().cpu() - (ref - c64)).abs().max().item()
    assert e1 <= 2 * ULP[dt] * (ref - c64).abs().max().item(), (tag, e1)
    dims = tuple(range(ref.dim() - 1))
    sd = ref.std(dim=dims)

    def bn_err(d):
        return (d.pow(2).mean(dim=dims).sqrt() / sd).mean().item()
    err_c = bn_err(y1.double().cpu() + c64 - ref)
    err_u = bn_err(y0.double().cpu() - ref)
    assert err_c < 0.5 * err_u, (tag, err_c, err_u)
    return err_c, err_u


@pytest.mark.parametrize("dt", DTYPES, ids=["bf16", "f16"])
@pytest.mark.parametrize("case", ROUTES, ids=lambda c: f"{c[0]}-K{c[4]}-N{c[5]}-R{c[6]}s{c[7]}")
def test_centred_store_every_forward_route(case, dt):
    from mauv import ops
    route, G, B, H, Cin, Cout, R, st, pd = case
    x, w = _large_mean_operands(G, B, H, Cin, Cout, R, dt)
    ref = _ref(x, w, st, pd)
    # the centre: the channel mean of the truth, moved a little (a running mean lags the batch)
    c = (ref.mean(dim=(0, 1, 2, 3)) * 1.01).float().to(dev).contiguous()
    xd, wd = x.to(dev), w.to(dev)
    Ho = ops.out_hw(H, R, st, pd)
    prev = ops.set_route(**ROUTE_SET[route])
    try:
        outs = []
        for ysh in (None, c):
            y = torch.full((G, B, Ho, Ho, Cout), float("nan"), device=dev, dtype=dt)
            stats = _stat_bufs(ops, G, B, H, Cin, Cout, R, st, pd)
            ops.conv2d_fwd(xd, wd, y, G, B, H, H, Cin, Cout, R, st, pd, stats=stats, ysh=ysh)
            torch.cuda.synchronize()
            outs.append((y, stats))
    finally:
        ops.set_route(**prev)
    (y0, s0), (y1, s1) = outs
    assert not torch.isnan(y1).any()
    _check_stats(s0, s1, c)
    ec, eu = _check_centred(y0, y1, c, ref, dt, route)
    # the same centre through the implicit GEMM: bit-identical where the route keeps its k order
    # (haloc16 runs 64-channel chunks outer, taps inner: fp32-summation close, checked above)
    if route not in ("pipe16", "haloc16"):
        prev = ops.set_route(**ROUTE_SET["pipe16"])
        try:
            yp = torch.full_like(y1, float("nan"))
            sp = _stat_bufs(ops, G, B, H, Cin, Cout, R, st, pd)
            ops.conv2d_fwd(xd, wd, yp, G, B, H, H, Cin, Cout, R, st, pd, stats=sp, ysh=c)
            torch.cuda.synchronize()
        finally:
            ops.set_route(**prev)
        assert torch.equal(yp, y1), route
        for a_, b_ in zip(sp, s1):
            assert torch.equal(a_, b_), route
    print(f"\n{route} {str(dt)[6:]} K={Cin * R * R} N={Cout}: rms error / channel std, centred "
          f"{ec:.3e} uncentred {eu:.3e}")


@pytest.mark.parametrize("dt", DTYPES, ids=["bf16", "f16"])
def test_centred_store_stem_and_fold(dt):
    from mauv import ops
    G, B, H, C = 2, 2, 32, 3
    g = torch.Generator().manual_seed(3)
    x = torch.rand(B, C, H, H, generator=g)
    K = C * 49
    Kp = ops.stem_kp(dt, K)
    Ho = ops.out_hw(H, 7, 2, 3)
    M = B * Ho * Ho
    cols = torch.empty(M, Kp, device=dev, dtype=dt)
    ops.stem_im2col(x.to(dev), B, C, H, H, 7, 2, 3, Kp, cols)
    w = torch.zeros(G, 64, Kp)
    w[..., :K] = torch.randn(G, 64, K, generator=g) / math.sqrt(K) + 0.02
    w = w.to(dt).to(dev)
    ref = torch.einsum("mk,gnk->gmn", cols.double(), w.double()).reshape(G, B, Ho, Ho, 64)
    c = (ref.mean(dim=(0, 1, 2, 3)) * 0.99).float().contiguous()
    outs = []
    for ysh in (None, c):
        y = torch.full((G, B, Ho, Ho, 64), float("nan"), device=dev, dtype=dt)
        nblk = ops.fwd_stat_blocks(G, B, H, H, C, 64, 7, 2, 3)
        stats = tuple(torch.full(s, float("nan"), device=dev) for s in
                      ((G, nblk, 64), (G, nblk, 64), (G, nblk)))
        ops.stem_fwd(cols, w, y, G, M, Kp, 64, stats, K, ysh=ysh)
        torch.cuda.synchronize()
        outs.append((y, stats))
    (y0, s0), (y1, s1) = outs
    _check_stats(s0, s1, c)
    _check_centred(y0, y1, c, ref, dt, "stem")
    # the fold: the block output it writes through is untouched by the centre; y1 centred
    Gf, Bf, Hf, Cin, Cout = 2, 2, 16, 256, 128
    torch.manual_seed(5)
    y3 = torch.randn(Gf, Bf, Hf, Hf, Cin).to(dt).to(dev)
    res = torch.rand(Gf, Bf, Hf, Hf, Cin).to(dt).to(dev)
    sc = (torch.rand(Gf, Cin) + 0.5).to(dev)
    sh = (torch.rand(Gf, Cin) + 0.5).to(dev)
    wf = ((torch.randn(Gf, Cout, 1, 1, Cin) + 0.3) / math.sqrt(Cin)).to(dt).to(dev)
    outs = []
    for ysh in (None, "c"):
        out = torch.full_like(y3, float("nan"))
        y1f = torch.full((Gf, Bf, Hf, Hf, Cout), float("nan"), device=dev, dtype=dt)
        nblk = ops.fwd_stat_blocks(Gf, Bf, Hf, Hf, Cin, Cout, 1, 1, 0)
        stats = tuple(torch.full(s, float("nan"), device=dev) for s in
                      ((Gf, nblk, Cout), (Gf, nblk, Cout), (Gf, nblk)))
        if ysh == "c":
            blk = outs[0][0].double()
            reff = torch.einsum("gmk,gnk->gmn", blk.reshape(Gf, -1, Cin),
                                wf.double().reshape(Gf, Cout, Cin)).reshape(Gf, Bf, Hf, Hf, Cout)
            cf = (reff.mean(dim=(0, 1, 2, 3)) * 1.01).float().contiguous()
        assert ops.conv2d_fwd_fold(y3, sc, sh, res, None, out, wf, y1f, Gf, Bf, Hf, Hf, Cin,
                                   Cout, stats=stats, ysh=None if ysh is None else cf)
        torch.cuda.synchronize()
        outs.append((out, y1f, stats))
    (o0, f0, t0), (o1, f1, t1) = outs
    assert torch.equal(o0, o1)
    _check_stats(t0, t1, cf.to(dev))
    _check_centred(f0, f1, cf, reff, dt, "fold")


@pytest.mark.parametrize("nblk", [7, 20000], ids=["one-launch", "segmented"])
def test_finalize_with_centre(nblk):
    from mauv import ops
    G, C = 3, 96
    g = torch.Generator().manual_seed(11)
    pm = (torch.randn(G, nblk, C, generator=g) * 0.1 + 40.0).to(dev)   # partial means of y
    p2 = (torch.rand(G, nblk, C, generator=g) * 5 + 1).to(dev)
    pc = torch.full((G, nblk), 128.0, device=dev)
    gamma = (torch.rand(C, generator=g) + 0.5).to(dev)
    beta = (torch.randn(C, generator=g) * 0.1).to(dev)
    rm0 = (torch.randn(C, generator=g) + 40.0).to(dev)
    rv0 = (torch.rand(C, generator=g) + 1).to(dev)

    def run(ysh_kind):
        rm, rv = rm0.clone(), rv0.clone()
        ws = torch.empty(ops.bn_stats_workspace_floats(G, nblk, C), device=dev)
        out = [torch.empty(G, C, device=dev) for _ in range(4)]
        ysh = None if ysh_kind is None else (rm if ysh_kind == "alias" else rm0.clone())
        # a centred forward's partials are those of the stored values y - c
        pmx = pm if ysh_kind is None else pm - rm0.view(1, 1, -1)
        ops.bn_stats_finalize(G, nblk, C, pmx, p2, pc, gamma, beta, rm, rv, 0.1, 1e-5, ws, *out,
                              ysh=ysh)
        torch.cuda.synchronize()
        return out, rm, rv
    (m0, i0, s0, h0), rm_a, rv_a = run(None)
    (m1, i1, s1, h1), rm_b, rv_b = run("copy")
    (m2, i2, s2, h2), rm_c, rv_c = run("alias")
    # the spread does not move (the merge of shifted partial means rounds differently)
    assert torch.allclose(i1, i0, rtol=1e-5, atol=0) and torch.allclose(s1, s0, rtol=1e-5, atol=0)
    assert torch.equal(m1, m2) and torch.equal(h1, h2) and torch.equal(rm_b, rm_c) and \
        torch.equal(rv_b, rv_c)                                # aliasing run_mean is safe
    assert torch.allclose(m1, m0 - rm0, atol=1e-5, rtol=0)    # the stored values' mean
    assert torch.allclose(rm_b, rm_a, atol=1e-5, rtol=0) and torch.allclose(rv_b, rv_a, rtol=1e-5)
    # a stored value v = y - c maps to the same normalised output as y did
    y = torch.randn(G, C, device=dev) * 2 + 40
    assert torch.allclose((y - rm0) * s1 + h1, y * s0 + h0, atol=1e-4, rtol=2e-6)
