"""16-bit (bf16 / f16) implicit-GEMM convs vs a float64 reference on the SAME 16-bit-rounded
operands: differences come only from fp32 accumulation order and the final rounding of the
16-bit outputs (tolerance: 2 ulp of the output format relative to max|ref|; fp32 weight-
gradient slabs 1e-4)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

dev = "cuda"
DTYPES = [torch.bfloat16, torch.float16]
ULP = {torch.bfloat16: 2.0 ** -8, torch.float16: 2.0 ** -11}


def close(a, b, rtol, atol=0.0):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    err = (a - b).abs().max().item()
    lim = atol + rtol * b.abs().max().item()
    assert err <= lim, f"max err {err:.3e} > {lim:.3e}"


def ref_conv(x, w, stride, pad):
    outs = []
    for g in range(w.shape[0]):
        xg = x[g if x.shape[0] > 1 else 0].permute(0, 3, 1, 2).double()
        outs.append(F.conv2d(xg, w[g].permute(0, 3, 1, 2).double(), stride=stride,
                             padding=pad).permute(0, 2, 3, 1))
    return torch.stack(outs)


CASES = [
    # G, B, H, Cin, Cout, R, stride, pad
    (2, 2, 8, 64, 64, 1, 1, 0),
    (2, 2, 8, 64, 64, 3, 1, 1),
    (2, 3, 9, 128, 128, 3, 2, 1),
    (1, 2, 8, 256, 512, 1, 2, 0),
    (2, 2, 4, 512, 2048, 1, 1, 0),
    (3, 2, 5, 64, 256, 1, 1, 0),
    (2, 2, 7, 8, 64, 3, 1, 1),      # Cin % 32 != 0: per-chunk tap decomposition, K tail
    (1, 4, 20, 64, 128, 3, 1, 1),   # 128 x 128 eight-wave tiles, ragged last m tile
    (2, 2, 15, 128, 64, 3, 2, 1),   # strided dgrad with Cout = 64, odd extents
    (1, 2, 6, 96, 64, 3, 1, 1),     # Cin % 64 != 0: the pipelined FWD declines, DGRAD/WGRAD run
    (1, 2, 12, 256, 256, 3, 1, 1),  # N >= 256, M > 64: two 128-wide n tiles (fwd, dgrad)
    (2, 3, 9, 64, 512, 1, 1, 0),    # 128 x 128 fwd tiles, ragged m, four n tiles; K = 64:
                                    # the one-stage forward kernel
    (2, 3, 9, 128, 256, 1, 1, 0),   # K = 128 / 256: the short-K sequential forward kernel
    (1, 3, 10, 256, 256, 1, 1, 0),
    (2, 3, 9, 128, 64, 1, 1, 0),    # dgrad over a single 64-deep stage: the one-stage kernel
    (2, 3, 9, 256, 128, 1, 1, 0),   # dgrad K = 128: the short-K sequential data gradient
]


@pytest.mark.parametrize("dt", DTYPES, ids=["bf16", "f16"])
@pytest.mark.parametrize("case", CASES)
def test_conv16_fwd_dgrad_wgrad(case, dt):
    from mauv import ops
    G, B, H, Cin, Cout, R, st, pad = case
    torch.manual_seed(0)
    x = torch.randn(G, B, H, H, Cin).to(dt)
    w = (torch.randn(G, Cout, R, R, Cin) / math.sqrt(Cin * R * R)).to(dt)
    Ho = ops.out_hw(H, R, st, pad)
    y = torch.empty(G, B, Ho, Ho, Cout, device=dev, dtype=dt)
    ops.conv2d_fwd(x.to(dev), w.to(dev), y, G, B, H, H, Cin, Cout, R, st, pad)
    close(y, ref_conv(x, w, st, pad), 2 * ULP[dt])

    dy = torch.randn(G, B, Ho, Ho, Cout).to(dt)
    dx_ref, dw_ref = [], []
    for g in range(G):
        xg = x[g].permute(0, 3, 1, 2).double().requires_grad_(True)
        wg = w[g].permute(0, 3, 1, 2).double().requires_grad_(True)
        F.conv2d(xg, wg, stride=st, padding=pad).backward(dy[g].permute(0, 3, 1, 2).double())
        dx_ref.append(xg.grad.permute(0, 2, 3, 1))
        dw_ref.append(wg.grad.permute(0, 2, 3, 1))
    if Cout % 32 == 0:
        addend = torch.randn(G, B, H, H, Cin).to(dt)
        dx = torch.empty(G, B, H, H, Cin, device=dev, dtype=dt)
        ops.conv2d_bwd_data(dy.to(dev), w.to(dev), dx, G, B, H, H, Cin, Cout, R, st, pad,
                            addend=addend.to(dev))
        close(dx, torch.stack(dx_ref) + addend.double(), 4 * ULP[dt])
    splits = ops.wgrad_splits(G, B, H, H, Cin, Cout, R, st, pad)
    ws = torch.empty(splits, G, Cout, R * R * Cin, device=dev)
    ops.conv2d_bwd_weight(x.to(dev), dy.to(dev), ws, splits, G, B, H, H, Cin, Cout, R, st, pad)
    close(ws.sum(0).view(G, Cout, R, R, Cin), torch.stack(dw_ref), 1e-4)


@pytest.mark.parametrize("dt", DTYPES, ids=["bf16", "f16"])
def test_conv16_stem_shared_padded_input(dt):
    """7x7/2 stem on a G-shared NHWC input whose 3 channels are zero-padded to 8."""
    from mauv import ops
    G, B, H, cin = 3, 2, 20, 3
    torch.manual_seed(1)
    x = torch.zeros(1, B, H, H, 8)
    x[..., :cin] = torch.randn(1, B, H, H, cin)
    x = x.to(dt)
    w = torch.zeros(G, 64, 7, 7, 8)
    w[..., :cin] = torch.randn(G, 64, 7, 7, cin) * 0.1
    w = w.to(dt)
    Ho = ops.out_hw(H, 7, 2, 3)
    strides = (0, H * H * 8, H * 8, 8, 1)
    y = torch.empty(G, B, Ho, Ho, 64, device=dev, dtype=dt)
    xd = x.to(dev)
    ops.conv2d_fwd(xd, w.to(dev), y, G, B, H, H, 8, 64, 7, 2, 3, x_strides=strides)
    close(y, ref_conv(x, w, 2, 3), 2 * ULP[dt])
    dy = torch.randn(G, B, Ho, Ho, 64).to(dt)
    splits = ops.wgrad_splits(G, B, H, H, 8, 64, 7, 2, 3)
    ws = torch.empty(splits, G, 64, 49 * 8, device=dev)
    ops.conv2d_bwd_weight(xd, dy.to(dev), ws, splits, G, B, H, H, 8, 64, 7, 2, 3,
                          x_strides=strides)
    ref = []
    for g in range(G):
        wg = w[g].permute(0, 3, 1, 2).double().requires_grad_(True)
        F.conv2d(x[0].permute(0, 3, 1, 2).double(), wg, stride=2, padding=3).backward(
            dy[g].permute(0, 3, 1, 2).double())
        ref.append(wg.grad.permute(0, 2, 3, 1))
    close(ws.sum(0).view(G, 64, 7, 7, 8), torch.stack(ref), 1e-4)


@pytest.mark.parametrize("dt", DTYPES, ids=["bf16", "f16"])
@pytest.mark.parametrize("Cout", [128, 256])
@pytest.mark.parametrize("Cin,R", [(64, 3), (64, 1), (128, 1)])
def test_conv16_lazy_bn_input_and_stats(dt, Cout, Cin, R):
    """x' = relu(x*scale + shift) applied on load (FWD and WGRAD) + epilogue statistics
    (3x3: the two-stage pipeline; 1x1 over 64 / 128 channels: the one-stage and short-K
    forward kernels)."""
    from mauv import ops
    G, B, H = 2, 3, 8
    torch.manual_seed(3)
    x = torch.randn(G, B, H, H, Cin).to(dt)
    sc = torch.rand(G, Cin) + 0.5
    sh = torch.randn(G, Cin) * 0.3
    pd = R // 2
    w = (torch.randn(G, Cout, R, R, Cin) / (8 * R)).to(dt)
    xt = torch.relu(x.float() * sc[:, None, None, None] + sh[:, None, None, None]).to(dt)
    ref = ref_conv(xt, w, 1, pd)
    nblk = ops.fwd_stat_blocks(G, B, H, H, Cin, Cout, R, 1, pd)
    pm = torch.empty(G, nblk, Cout, device=dev)
    pm2 = torch.empty_like(pm)
    pc = torch.empty(G, nblk, device=dev)
    y = torch.empty(G, B, H, H, Cout, device=dev, dtype=dt)
    ops.conv2d_fwd(x.to(dev), w.to(dev), y, G, B, H, H, Cin, Cout, R, 1, pd,
                   x_bn=(sc.to(dev), sh.to(dev), 1), stats=(pm, pm2, pc))
    close(y, ref, 2 * ULP[dt])
    # merged partials = mean / M2 of the fp32 (pre-rounding) output
    n = pc.double().cpu()
    mu = (pm.double().cpu() * n[..., None]).sum(1) / n.sum(1, keepdim=True)
    m2 = (pm2.double().cpu() + n[..., None] * (pm.double().cpu() - mu[:, None]) ** 2).sum(1)
    r = ref.reshape(G, -1, Cout)
    close(mu, r.mean(1), 1e-4)
    close(m2 / r.shape[1], r.var(1, unbiased=False), 1e-3)
    dy = torch.randn(G, B, H, H, Cout).to(dt)
    splits = ops.wgrad_splits(G, B, H, H, Cin, Cout, R, 1, pd)
    ws = torch.empty(splits, G, Cout, R * R * Cin, device=dev)
    ops.conv2d_bwd_weight(x.to(dev), dy.to(dev), ws, splits, G, B, H, H, Cin, Cout, R, 1, pd,
                          x_bn=(sc.to(dev), sh.to(dev), 1))
    dw = []
    for g in range(G):
        wg = w[g].permute(0, 3, 1, 2).double().requires_grad_(True)
        F.conv2d(xt[g].permute(0, 3, 1, 2).double(), wg, padding=pd).backward(
            dy[g].permute(0, 3, 1, 2).double())
        dw.append(wg.grad.permute(0, 2, 3, 1))
    close(ws.sum(0).view(G, Cout, R, R, Cin), torch.stack(dw), 1e-3)


@pytest.mark.parametrize("dt", DTYPES, ids=["bf16", "f16"])
@pytest.mark.parametrize("C,relu,res,lazy", [(64, True, False, True), (256, True, True, False),
                                             (2048, False, False, False)])
def test_bn16_apply_bwd_matches_fp32_kernels(dt, C, relu, res, lazy):
    """16-bit BN apply / backward == the fp32 kernels on the same 16-bit-rounded tensors, up
    to the final rounding of the 16-bit outputs."""
    from mauv import ops
    G, M = 3, 4 * 5 * 5
    torch.manual_seed(5)
    y = (torch.randn(G, M, C) * 3 + 2).to(dt).to(dev)
    r = torch.randn(G, M, C).to(dt).to(dev) if res else None
    dout = torch.randn(G, M, C).to(dt).to(dev)
    mean = y.float().mean(1)
    invstd = (y.float().var(1, unbiased=False) + 1e-5).rsqrt()
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev)
    scale = (gamma * invstd).contiguous()
    shift = (beta - mean * scale).contiguous()
    out16 = torch.empty(G, M, C, device=dev, dtype=dt)
    ops.bn_apply(y, scale, shift, r, relu, out16, G, M, C)
    out32 = torch.empty(G, M, C, device=dev)
    ops.bn_apply(y.float(), scale, shift, None if r is None else r.float(), relu, out32, G, M, C)
    close(out16, out32, 2 * ULP[dt])
    ws = torch.empty(ops.bn_workspace_floats(G, M, C), device=dev)
    res16 = [torch.empty(G, M, C, device=dev, dtype=dt), torch.empty(G, M, C, device=dev, dtype=dt)
             if res else None, torch.zeros(C, device=dev), torch.zeros(C, device=dev)]
    res32 = [torch.empty(G, M, C, device=dev), torch.empty(G, M, C, device=dev) if res else None,
             torch.zeros(C, device=dev), torch.zeros(C, device=dev)]
    o16 = None if lazy else out16
    o32 = None if lazy else out16.float()   # the same (rounded) mask source
    ops.bn_bwd(y, o16, dout, relu, mean, invstd, scale, G, M, C, ws, *res16, shift=shift)
    ws2 = torch.empty_like(ws)
    ops.bn_bwd(y.float(), o32, dout.float(), relu, mean, invstd, scale, G, M, C, ws2, *res32,
               shift=shift)
    close(res16[0], res32[0], 4 * ULP[dt])
    if res:
        close(res16[1], res32[1], 2 * ULP[dt])
    close(res16[2], res32[2], 1e-5)
    close(res16[3], res32[3], 1e-5)


@pytest.mark.parametrize("dt", DTYPES, ids=["bf16", "f16"])
@pytest.mark.parametrize("N,H,C", [(2, 10, 12), (5, 16, 64), (1, 7, 8)])
def test_maxpool16_bwd_shapes(dt, N, H, C):
    """8-channel gather (C % 8 == 0) and the 4-channel one (C = 12), even / odd sizes: the max-pool
    backward equals autograd of F.max_pool2d on the same argmax (no ties: distinct values)."""
    from mauv import ops
    torch.manual_seed(16 + C)
    x = (torch.randperm(N * H * H * C).float() / 64.0).reshape(N, H, H, C).to(dt)
    Ho = ops.out_hw(H, 3, 2, 1)
    xr = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    yr, flat = F.max_pool2d(xr, 3, 2, 1, return_indices=True)
    # the argmax as the kernels store it: tap r*3 + s of the window at (2*oh - 1, 2*ow - 1)
    oh = torch.arange(Ho).view(1, 1, Ho, 1)
    ow = torch.arange(Ho).view(1, 1, 1, Ho)
    tap = (flat // H - (2 * oh - 1)) * 3 + (flat % H - (2 * ow - 1))
    idx_ref = tap.permute(0, 2, 3, 1).to(torch.uint8).contiguous()
    if C % 8 == 0:   # the 16-bit forward (8-channel chunks) writes the same argmax bytes
        y = torch.empty(N, Ho, Ho, C, device=dev, dtype=dt)
        idx = torch.empty(N, Ho, Ho, C, dtype=torch.uint8, device=dev)
        ops.maxpool_fwd(x.to(dev), N, H, H, C, y, idx)
        assert torch.equal(idx.cpu(), idx_ref)
    dy = torch.randn(N, Ho, Ho, C).to(dt)
    yr.backward(dy.double().permute(0, 3, 1, 2))
    dx = torch.empty(N, H, H, C, device=dev, dtype=dt)
    ops.maxpool_bwd(dy.to(dev), idx_ref.to(dev), N, H, H, C, dx)
    close(dx, xr.grad.permute(0, 2, 3, 1), 2 * ULP[dt])


@pytest.mark.parametrize("dt", DTYPES, ids=["bf16", "f16"])
def test_pools16_and_stem_pack(dt):
    from mauv import ops
    N, H, C = 3, 9, 64
    torch.manual_seed(6)
    x = torch.randn(N, H, H, C).to(dt)
    x[0, :3, :3, :] = 0.0
    Ho = ops.out_hw(H, 3, 2, 1)
    y = torch.empty(N, Ho, Ho, C, device=dev, dtype=dt)
    idx = torch.empty(N, Ho, Ho, C, dtype=torch.uint8, device=dev)
    ops.maxpool_fwd(x.to(dev), N, H, H, C, y, idx)
    xr = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    close(y, yr.permute(0, 2, 3, 1), 0.0)          # max is exact
    dy = torch.randn(N, Ho, Ho, C).to(dt)
    yr.backward(dy.double().permute(0, 3, 1, 2))
    dx = torch.empty(N, H, H, C, device=dev, dtype=dt)
    ops.maxpool_bwd(dy.to(dev), idx, N, H, H, C, dx)
    close(dx, xr.grad.permute(0, 2, 3, 1), 2 * ULP[dt])
    a = torch.empty(N, C, device=dev)
    ops.avgpool_fwd(x.to(dev), N, H * H, C, a)
    close(a, x.double().mean((1, 2)), 1e-5)
    da = torch.randn(N, C)
    dxa = torch.empty(N, H, H, C, device=dev, dtype=dt)
    ops.avgpool_bwd(da.to(dev), N, H * H, C, dxa)
    close(dxa, (da.double() / (H * H))[:, None, None, :].expand(N, H, H, C), 2 * ULP[dt])
    img = torch.randn(2, 3, 7, 5)
    packed = torch.empty(2, 7, 5, 8, device=dev, dtype=dt)
    ops.pack_nchw(img.to(dev), 2, 3, 7, 5, 8, packed)
    ref = torch.zeros(2, 7, 5, 8)
    ref[..., :3] = img.permute(0, 2, 3, 1)
    assert torch.equal(packed.cpu(), ref.to(dt))


@pytest.mark.parametrize("dt", DTYPES, ids=["bf16", "f16"])
def test_reparam16_padded_sample_and_bwd(dt):
    """16-bit sampled weights (cin padded 3 -> 8) == round(fp32 sample); reparam_bwd over
    padded slabs == over dense slabs."""
    from mauv import ops
    G, Cout, Cin, RS, cp = 3, 16, 3, 49, 8
    torch.manual_seed(7)
    mu = torch.randn(Cout, Cin, RS, device=dev) * 0.1
    rho = torch.randn(Cout, Cin, RS, device=dev) - 3
    w32 = torch.empty(G, Cout, RS, Cin, device=dev)
    ops.reparam_sample(mu, rho, w32, G, 42, 5, 9, Cout, Cin, RS)
    w16 = torch.zeros(G, Cout, RS, cp, device=dev, dtype=dt)
    ops.reparam_sample(mu, rho, w16, G, 42, 5, 9, Cout, Cin, RS, cin_pad=cp)
    assert torch.equal(w16[..., :Cin], w32.to(dt)) and not w16[..., Cin:].any()
    dwp = torch.zeros(2, G, Cout, RS, cp, device=dev)
    dwp[..., :Cin] = torch.randn(2, G, Cout, RS, Cin, device=dev)
    dwp[..., Cin:] = 1e9    # padded channels must be ignored
    dmu_a, drho_a = torch.zeros_like(mu), torch.zeros_like(rho)
    ops.reparam_bwd(dwp, 2, mu, rho, dmu_a, drho_a, G, 42, 5, 9, Cout, Cin, RS, dw_cin=cp)
    dmu_b, drho_b = torch.zeros_like(mu), torch.zeros_like(rho)
    ops.reparam_bwd(dwp[..., :Cin].contiguous(), 2, mu, rho, dmu_b, drho_b, G, 42, 5, 9, Cout,
                    Cin, RS)
    assert torch.equal(dmu_a, dmu_b) and torch.equal(drho_a, drho_b)



@pytest.mark.parametrize("dt", DTYPES + [torch.float32], ids=["bf16", "f16", "fp32"])
@pytest.mark.parametrize("case,src,res", [
    ((2, 2, 8, 64, 64, 3, 1, 1), "lazy", False),       # bn1/bn2 of a block: mask from y*sc+sh
    ((1, 3, 9, 128, 128, 3, 2, 1), "lazy", False),     # strided: four parity classes, ragged
    ((2, 3, 9, 256, 64, 1, 1, 0), "mask", True),       # block output: mask bits + residual addend
    ((2, 2, 15, 64, 128, 3, 2, 1), "out", False),      # BN 64-wide column tiles, odd extents
    ((1, 2, 4, 512, 2048, 1, 1, 0), "none", True),     # no ReLU (the downsample's BN), BM = 64
    ((1, 8, 136, 64, 64, 1, 1, 0), "mask", True),      # 1,156 partials per channel: the
                                                       # segmented finalize (bn_bwd_seg)
    ((2, 2, 12, 512, 128, 1, 1, 0), "mask", True),     # 16-bit: the short-K form (K = 128)
    ((1, 2, 12, 1024, 256, 1, 1, 0), "lazy", False),   # 16-bit: the short-K form (K = 256)
])
def test_conv16_dgrad_bn_partials_epilogue(case, src, res, dt):
    """The data gradient's epilogue writes the BN-backward partials of the BN whose output
    gradient dx is (conv2d_bwd_data(..., bn=...); 16-bit: conv_epi16.h, fp32: the split
    kernel's LDS-staged epilogue, conv_common.h staged_epilogue_f32): dx bit-identical to the plain data gradient;
    the BN backward finished from those partials (bn_bwd_ex(pre=...)) matches the standalone
    partial pass within fp32 summation order, and both match float64 on the same 16-bit dx."""
    from mauv import ops
    G, B, H, Cin, Cout, R, st, pad = case
    torch.manual_seed(5)
    Ho = ops.out_hw(H, R, st, pad)
    C, M = Cin, B * H * H
    dyc = (torch.randn(G, B, Ho, Ho, Cout) * 0.5).to(dt).to(dev)
    w = (torch.randn(G, Cout, R, R, Cin) / math.sqrt(Cin * R * R)).to(dt).to(dev)
    y = torch.randn(G, B, H, H, C).to(dt).to(dev)
    mean = (torch.randn(G, C) * 0.1).to(dev)
    invstd = (torch.rand(G, C) + 0.5).to(dev)
    sc = (torch.rand(G, C) + 0.5).to(dev)
    sh = (torch.randn(G, C) * 0.1).to(dev)
    addend = torch.randn(G, B, H, H, C).to(dt).to(dev) if res else None
    relu = src != "none"
    out = mask = None
    if src in ("out", "mask"):
        out = torch.empty_like(y)
        mask = torch.empty(G * M * C // 8, dtype=torch.uint8, device=dev)
        ops.bn_apply_mask(y, sc, sh, None, out, mask, G, M, C)
        if src == "mask":
            out = None
        else:
            mask = None
    dx_plain = torch.empty(G, B, H, H, C, device=dev, dtype=dt)
    ops.conv2d_bwd_data(dyc, w, dx_plain, G, B, H, H, Cin, Cout, R, st, pad, addend=addend)
    nblk = ops.dgrad_stat_blocks(G, B, H, H, Cin, Cout, R, st, pad)
    p1 = torch.full((G, nblk, C), float("nan"), device=dev)
    p2 = torch.full((G, nblk, C), float("nan"), device=dev)
    dx = torch.empty_like(dx_plain)
    bn = dict(y=y, out=out, mask=mask, scale=sc, shift=sh, mean=mean, invstd=invstd, relu=relu,
              p1=p1, p2=p2)
    ops.conv2d_bwd_data(dyc, w, dx, G, B, H, H, Cin, Cout, R, st, pad, addend=addend, bn=bn)
    torch.cuda.synchronize()
    assert torch.equal(dx, dx_plain)
    assert torch.isfinite(p1).all() and torch.isfinite(p2).all()    # every block written
    ws = torch.empty(ops.bn_workspace_floats(G, M, C), device=dev)
    res_ = {}
    for key, pre in (("epi", (p1, p2, nblk)), ("pass", None)):
        dyo = torch.empty_like(y)
        dg = torch.zeros(C, device=dev)
        db = torch.zeros(C, device=dev)
        ops.bn_bwd_ex(y, out, mask, dx, relu, mean, invstd, sc, sh, G, M, C, ws, dyo,
                      dgamma=dg, dbeta=db, pre=pre)
        res_[key] = (dyo, dg, db)
    # float64 truth on the same 16-bit dx
    yd, dd = y.double().view(G, M, C), dx.double().view(G, M, C)
    if relu:
        pre_act = (out.double().view(G, M, C) if out is not None else
                   (y.double().view(G, M, C) * sc.double()[:, None] + sh.double()[:, None]))
        if mask is not None:     # the bits are of the stored (rounded) output
            o16 = torch.empty_like(y)
            ops.bn_apply(y, sc, sh, None, True, o16, G, M, C)
            pre_act = o16.double().view(G, M, C)
        dz = dd * (pre_act > 0)
    else:
        dz = dd
    xh = (yd - mean.double()[:, None]) * invstd.double()[:, None]
    dbeta_t, dgamma_t = dz.sum((0, 1)), (dz * xh).sum((0, 1))
    for key in ("epi", "pass"):
        dyo, dg, db = res_[key]
        close(db, dbeta_t, 1e-4, 1e-3)
        close(dg, dgamma_t, 1e-4, 1e-3)
    close(res_["epi"][0], res_["pass"][0], 2 * ULP.get(dt, 2.0 ** -20))
    close(res_["epi"][1], res_["pass"][1], 1e-5, 1e-4)
    close(res_["epi"][2], res_["pass"][2], 1e-5, 1e-4)
