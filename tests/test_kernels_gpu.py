"""Kernel-level parity on the GPU: every libmauv_hip kernel vs a float64 torch-CPU
reference of the same op (conv fwd/dgrad/wgrad, BN fwd/bwd, pooling, reparam, KL, head).
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

dev = "cuda"


def close(a, b, rtol=1e-4, atol=1e-5):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    err = (a - b).abs().max().item()
    lim = atol + rtol * b.abs().max().item()
    assert err <= lim, f"max err {err:.3e} > {lim:.3e}"


CONV_CASES = [
    # G, B, H, Cin, Cout, R, stride, pad
    (2, 2, 8, 64, 64, 1, 1, 0),
    (2, 2, 8, 64, 64, 3, 1, 1),
    (2, 3, 9, 128, 128, 3, 2, 1),
    (1, 2, 8, 256, 512, 1, 2, 0),
    (2, 2, 4, 512, 2048, 1, 1, 0),
    (3, 2, 5, 64, 256, 1, 1, 0),
    (2, 3, 9, 64, 256, 1, 1, 0),     # 1x1 forwards with K <= 256 on 128 x 128 tiles: the
    (1, 3, 10, 256, 128, 1, 1, 0),   # split kernel's short-K (SEQ) variant (dgrad: K = 128)
    (2, 3, 9, 128, 64, 1, 1, 0),     # SEQ data gradient over K = 64
]


def _ref_conv(x, w, stride, pad):
    # x [G,B,H,W,C] w [G,Cout,R,R,Cin] -> y [G,B,Ho,Wo,Cout] (float64)
    outs = []
    for g in range(x.shape[0]):
        xg = x[g].permute(0, 3, 1, 2).double()
        wg = w[g].permute(0, 3, 1, 2).double()
        outs.append(F.conv2d(xg, wg, stride=stride, padding=pad).permute(0, 2, 3, 1))
    return torch.stack(outs)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(case):
    from mauv import ops
    G, B, H, Cin, Cout, R, st, pad = case
    torch.manual_seed(0)
    x = torch.randn(G, B, H, H, Cin)
    w = torch.randn(G, Cout, R, R, Cin) / math.sqrt(Cin * R * R)
    Ho = ops.out_hw(H, R, st, pad)
    ref = _ref_conv(x, w, st, pad)
    y = torch.empty(G, B, Ho, Ho, Cout, device=dev)
    ops.conv2d_fwd(x.to(dev), w.to(dev), y, G, B, H, H, Cin, Cout, R, st, pad)
    close(y, ref)

    dy = torch.randn(G, B, Ho, Ho, Cout)
    dx_ref, dw_ref = [], []
    for g in range(G):
        xg = x[g].permute(0, 3, 1, 2).double().requires_grad_(True)
        wg = w[g].permute(0, 3, 1, 2).double().requires_grad_(True)
        out = F.conv2d(xg, wg, stride=st, padding=pad)
        out.backward(dy[g].permute(0, 3, 1, 2).double())
        dx_ref.append(xg.grad.permute(0, 2, 3, 1))
        dw_ref.append(wg.grad.permute(0, 2, 3, 1))
    dx = torch.empty(G, B, H, H, Cin, device=dev)
    addend = torch.randn(G, B, H, H, Cin)
    ops.conv2d_bwd_data(dy.to(dev), w.to(dev), dx, G, B, H, H, Cin, Cout, R, st, pad,
                        addend=addend.to(dev))
    close(dx, torch.stack(dx_ref) + addend.double())
    splits = ops.wgrad_splits(G, B, H, H, Cin, Cout, R, st, pad)
    ws = torch.empty(splits, G, Cout, R * R * Cin, device=dev)
    ops.conv2d_bwd_weight(x.to(dev), dy.to(dev), ws, splits, G, B, H, H, Cin, Cout, R, st, pad)
    close(ws.sum(0).view(G, Cout, R, R, Cin), torch.stack(dw_ref))


@pytest.mark.parametrize("Cin,R", [(64, 3), (64, 1), (128, 1), (256, 1)])
def test_conv_lazy_bn_input_and_stats(Cin, R):
    """fp32 convs with the producing BN + ReLU applied on load (FWD and WGRAD) and the
    epilogue statistics: the two-stage split kernel (3x3) and its short-K variant (1x1)."""
    from mauv import ops
    G, B, H, Cout = 2, 3, 8, 128
    pd = R // 2
    torch.manual_seed(4)
    x = torch.randn(G, B, H, H, Cin)
    sc = torch.rand(G, Cin) + 0.5
    sh = torch.randn(G, Cin) * 0.3
    w = torch.randn(G, Cout, R, R, Cin) / (8 * R)
    xt = torch.relu(x * sc[:, None, None, None] + sh[:, None, None, None])
    ref = _ref_conv(xt, w, 1, pd)
    nblk = ops.fwd_stat_blocks(G, B, H, H, Cin, Cout, R, 1, pd)
    pm = torch.empty(G, nblk, Cout, device=dev)
    pm2 = torch.empty_like(pm)
    pc = torch.empty(G, nblk, device=dev)
    y = torch.empty(G, B, H, H, Cout, device=dev)
    xbn = (sc.to(dev), sh.to(dev), 1)
    ops.conv2d_fwd(x.to(dev), w.to(dev), y, G, B, H, H, Cin, Cout, R, 1, pd, x_bn=xbn,
                   stats=(pm, pm2, pc))
    close(y, ref)
    n = pc.double().cpu()
    mu = (pm.double().cpu() * n[..., None]).sum(1) / n.sum(1, keepdim=True)
    m2 = (pm2.double().cpu() + n[..., None] * (pm.double().cpu() - mu[:, None]) ** 2).sum(1)
    r = ref.reshape(G, -1, Cout)
    close(mu, r.mean(1))
    close(m2 / r.shape[1], r.var(1, unbiased=False), rtol=1e-4)
    dy = torch.randn(G, B, H, H, Cout)
    splits = ops.wgrad_splits(G, B, H, H, Cin, Cout, R, 1, pd)
    ws = torch.empty(splits, G, Cout, R * R * Cin, device=dev)
    ops.conv2d_bwd_weight(x.to(dev), dy.to(dev), ws, splits, G, B, H, H, Cin, Cout, R, 1, pd,
                          x_bn=xbn)
    dw = []
    for g in range(G):
        wg = w[g].permute(0, 3, 1, 2).double().requires_grad_(True)
        F.conv2d(xt[g].permute(0, 3, 1, 2).double(), wg, padding=pd).backward(
            dy[g].permute(0, 3, 1, 2).double())
        dw.append(wg.grad.permute(0, 2, 3, 1))
    close(ws.sum(0).view(G, Cout, R, R, Cin), torch.stack(dw))


@pytest.mark.parametrize("cin", [3, 1])
def test_stem_nchw_shared_input(cin):
    """Stem 7x7/2 reading the caller's NCHW images directly, input shared by G groups."""
    from mauv import ops
    G, B, H = 3, 2, 20
    torch.manual_seed(1)
    x = torch.randn(B, cin, H, H)
    w = torch.randn(G, 64, 7, 7, cin) * 0.1
    Ho = ops.out_hw(H, 7, 2, 3)
    strides = (0, cin * H * H, H, 1, H * H)
    y = torch.empty(G, B, Ho, Ho, 64, device=dev)
    xd = x.to(dev)
    ops.conv2d_fwd(xd, w.to(dev), y, G, B, H, H, cin, 64, 7, 2, 3, x_strides=strides)
    xs = x.permute(0, 2, 3, 1).unsqueeze(0).expand(G, -1, -1, -1, -1)
    close(y, _ref_conv(xs, w, 2, 3))
    dy = torch.randn(G, B, Ho, Ho, 64)
    splits = ops.wgrad_splits(G, B, H, H, cin, 64, 7, 2, 3)
    ws = torch.empty(splits, G, 64, 49 * cin, device=dev)
    ops.conv2d_bwd_weight(xd, dy.to(dev), ws, splits, G, B, H, H, cin, 64, 7, 2, 3,
                          x_strides=strides)
    ref = []
    for g in range(G):
        wg = w[g].permute(0, 3, 1, 2).double().requires_grad_(True)
        F.conv2d(x.double(), wg, stride=2, padding=3).backward(dy[g].permute(0, 3, 1, 2).double())
        ref.append(wg.grad.permute(0, 2, 3, 1))
    close(ws.sum(0).view(G, 64, 7, 7, cin), torch.stack(ref))


@pytest.mark.parametrize("cin,H,R", [(3, 20, 7), (1, 37, 7), (3, 9, 3)])
def test_stem_packed_nhwc4(cin, H, R):
    """Stems on the packed layout (mauv_pack_nchw_f32: NHWC, channels zero-padded to 4) with
    4-channel padded weights (mauv_reparam_sample_padded): the split kernel's STEM mode."""
    from mauv import ops
    G, B, st, pd = 3, 2, 2, R // 2
    torch.manual_seed(2)
    x = torch.randn(B, cin, H, H)
    mu = torch.randn(64, cin, R, R) * 0.1
    rho = torch.full_like(mu, -4.0)
    eps = torch.randn(G, 64 * cin * R * R)
    xd = x.to(dev)
    xp = torch.empty(B, H, H, 4, device=dev)
    ops.pack_nchw(xd, B, cin, H, H, 4, xp)
    ref_xp = torch.zeros(B, H, H, 4)
    ref_xp[..., :cin] = x.permute(0, 2, 3, 1)
    assert torch.equal(xp.cpu(), ref_xp)
    w = torch.zeros(G, 64, R, R, 4, device=dev)
    ops.reparam_sample(mu.to(dev), rho.to(dev), w, G, 0, 0, 0, 64, cin, R * R, eps=eps.to(dev),
                       cin_pad=4)
    wref = mu.unsqueeze(0) + F.softplus(rho).unsqueeze(0) * eps.view(G, 64, cin, R, R)
    close(w[..., :cin], wref.permute(0, 1, 3, 4, 2), rtol=1e-6, atol=1e-7)
    assert torch.count_nonzero(w[..., cin:]) == 0
    Ho = ops.out_hw(H, R, st, pd)
    strides = (0, H * H * 4, H * 4, 4, 1)
    y = torch.empty(G, B, Ho, Ho, 64, device=dev)
    ops.conv2d_fwd(xp, w, y, G, B, H, H, 4, 64, R, st, pd, x_strides=strides, alg_cin=cin)
    wc = w.cpu()[..., :cin]
    xs = x.permute(0, 2, 3, 1).unsqueeze(0).expand(G, -1, -1, -1, -1)
    close(y, _ref_conv(xs, wc, st, pd))
    dy = torch.randn(G, B, Ho, Ho, 64)
    splits = ops.wgrad_splits(G, B, H, H, 4, 64, R, st, pd)
    ws = torch.empty(splits, G, 64, R * R * 4, device=dev)
    ops.conv2d_bwd_weight(xp, dy.to(dev), ws, splits, G, B, H, H, 4, 64, R, st, pd,
                          x_strides=strides, alg_cin=cin)
    ref = []
    for g in range(G):
        wg = wc[g].permute(0, 3, 1, 2).double().requires_grad_(True)
        F.conv2d(x.double(), wg, stride=st, padding=pd).backward(dy[g].permute(0, 3, 1, 2).double())
        ref.append(wg.grad.permute(0, 2, 3, 1))
    close(ws.sum(0).view(G, 64, R, R, 4)[..., :cin], torch.stack(ref))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16],
                         ids=["fp32", "bf16", "f16"])
@pytest.mark.parametrize("cin,H,G", [(3, 20, 3), (1, 37, 4), (3, 33, 1), (1, 9, 5), (2, 21, 2)])
def test_stem_im2col_gemm(dt, cin, H, G):
    """The stems as one GEMM over shared im2col rows (stem.hip): rows bit-exact against
    F.unfold, outputs / BN partials / weight gradient against float64 convolutions of the
    same (rounded) operands; G odd leaves a ragged 64-column tile of the stacked N."""
    from mauv import ops
    B, R, st, pd = 2, 7, 2, 3
    torch.manual_seed(5)
    x = torch.randn(B, cin, H, H)
    K = cin * R * R
    Kp = ops.stem_kp(dt, K)
    Ho = ops.out_hw(H, R, st, pd)
    M = B * Ho * Ho
    cols = torch.empty(M, Kp, device=dev, dtype=dt)
    ops.stem_im2col(x.to(dev), B, cin, H, H, R, st, pd, Kp, cols)
    ref_cols = torch.zeros(M, Kp)
    ref_cols[:, :K] = F.unfold(x, R, padding=pd, stride=st).transpose(1, 2).reshape(M, K)
    assert torch.equal(cols.cpu(), ref_cols.to(dt)), "im2col rows differ"
    mu = torch.randn(64, cin, R, R) * 0.1
    rho = torch.full_like(mu, -4.0)
    eps = torch.randn(G, mu.numel())
    w = torch.zeros(G, 64, Kp, device=dev, dtype=dt)
    ops.reparam_sample(mu.to(dev), rho.to(dev), w, G, 0, 0, 0, 64, K, 1, eps=eps.to(dev),
                       cin_pad=Kp)
    wref = (mu.view(1, 64, K) + F.softplus(rho).view(1, 64, K) * eps.view(G, 64, K))
    close(w[..., :K].float(), wref, rtol=4e-3 if dt != torch.float32 else 1e-6, atol=1e-7)
    assert torch.count_nonzero(w[..., K:]) == 0
    nblk = ops.fwd_stat_blocks(G, B, H, H, cin, 64, R, st, pd)
    stats = torch.empty(2 * G * nblk * 64 + G * nblk, device=dev)
    sm, s2 = stats[:G * nblk * 64], stats[G * nblk * 64:2 * G * nblk * 64]
    sn = stats[2 * G * nblk * 64:]
    y = torch.empty(G, B, Ho, Ho, 64, device=dev, dtype=dt)
    ops.stem_fwd(cols, w, y, G, M, Kp, 64, (sm, s2, sn), K)
    wc = w.cpu().double()[..., :K].view(G, 64, cin, R, R)
    xr = x.to(dt).double()
    ref = torch.stack([F.conv2d(xr, wc[g], stride=st, padding=pd).permute(0, 2, 3, 1)
                       for g in range(G)])
    tol = 1e-4 if dt == torch.float32 else 8e-3
    close(y.float(), ref, rtol=tol)
    # per-m-tile partials merged -> the batch mean / variance of every group's channels
    cnt = sn.view(G, nblk).double().cpu()
    pm = sm.view(G, nblk, 64).double().cpu()
    pm2 = s2.view(G, nblk, 64).double().cpu()
    mean = (pm * cnt[..., None]).sum(1) / cnt.sum(1, keepdim=True)
    m2 = (pm2 + cnt[..., None] * (pm - mean[:, None]) ** 2).sum(1)
    assert torch.equal(cnt.sum(1), torch.full((G,), float(M), dtype=torch.float64))
    rf = ref.view(G, M, 64)
    close(mean, rf.mean(1), rtol=tol, atol=1e-5)
    close(m2 / M, rf.var(1, unbiased=False), rtol=tol * 2)
    # weight gradient: 1x1 weight-gradient GEMM over the shared rows
    dy = torch.randn(G, B, Ho, Ho, 64).to(dt)
    splits = ops.wgrad_splits(G, M, 1, 1, Kp, 64, 1, 1, 0)
    ws = torch.empty(splits, G, 64, Kp, device=dev)
    ops.conv2d_bwd_weight(cols, dy.to(dev), ws, splits, G, M, 1, 1, Kp, 64, 1, 1, 0,
                          x_strides=(0, Kp, Kp, Kp, 1), alg_cin=K)
    dref = []
    for g in range(G):
        wg = wc[g].clone().requires_grad_(True)
        F.conv2d(xr, wg, stride=st, padding=pd).backward(dy[g].double().permute(0, 3, 1, 2))
        dref.append(wg.grad.reshape(64, K))
    dw = ws.sum(0)
    close(dw[..., :K], torch.stack(dref), rtol=1e-4 if dt == torch.float32 else 2e-3)
    assert torch.count_nonzero(dw[..., K:]) == 0


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
@pytest.mark.parametrize("R,st,pd", [(1, 2, 0), (3, 2, 1), (1, 1, 0)])
def test_dgrad_accumulate_into_dx(dt, R, st, pd):
    """dx += dgrad(dy, w) (the downsample branch adding into the main branch's dx): classes of a
    strided conv without taps leave dx untouched."""
    from mauv import ops
    G, B, H, Cin, Cout = 2, 2, 9, 64, 128
    torch.manual_seed(4)
    Ho = ops.out_hw(H, R, st, pd)
    dy = torch.randn(G, B, Ho, Ho, Cout).to(dt)
    w = (torch.randn(G, Cout, R, R, Cin) / (Cin * R * R) ** 0.5).to(dt)
    dx0 = torch.randn(G, B, H, H, Cin).to(dt)
    dx = dx0.to(dev).clone()
    ops.conv2d_bwd_data(dy.to(dev), w.to(dev), dx, G, B, H, H, Cin, Cout, R, st, pd,
                        accumulate=True)
    ref = []
    for g in range(G):
        xg = torch.zeros(B, Cin, H, H, dtype=torch.float64, requires_grad=True)
        F.conv2d(xg, w[g].permute(0, 3, 1, 2).double(), stride=st, padding=pd).backward(
            dy[g].permute(0, 3, 1, 2).double())
        ref.append(xg.grad.permute(0, 2, 3, 1))
    ref = torch.stack(ref) + dx0.double()
    tol = 1e-5 if dt == torch.float32 else 2 ** -7
    close(dx.float(), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("K,N", [(2048, 384), (384, 1284), (1284, 32), (32, 7), (128, 128)])
def test_linear_as_1x1(K, N):
    from mauv import ops
    G, B = 2, 5
    torch.manual_seed(2)
    x = torch.randn(G, B, K)
    w = torch.randn(G, N, K) / math.sqrt(K)
    b = torch.randn(G, N)
    y = torch.empty(G, B, N, device=dev)
    ops.conv2d_fwd(x.to(dev), w.to(dev), y, G, B, 1, 1, K, N, 1, 1, 0, bias=b.to(dev))
    ref = torch.einsum("gbk,gnk->gbn", x.double(), w.double()) + b.double()[:, None]
    close(y, ref)
    dy = torch.randn(G, B, N)
    dx = torch.empty(G, B, K, device=dev)
    ops.conv2d_bwd_data(dy.to(dev), w.to(dev), dx, G, B, 1, 1, K, N, 1, 1, 0)
    close(dx, torch.einsum("gbn,gnk->gbk", dy.double(), w.double()))
    splits = ops.wgrad_splits(G, B, 1, 1, K, N, 1, 1, 0)
    ws = torch.empty(splits, G, N, K, device=dev)
    ops.conv2d_bwd_weight(x.to(dev), dy.to(dev), ws, splits, G, B, 1, 1, K, N, 1, 1, 0)
    close(ws.sum(0), torch.einsum("gbn,gbk->gnk", dy.double(), x.double()))
    db = torch.empty(G, N, device=dev)
    ops.colsum(dy.to(dev), G, B, N, db)
    close(db, dy.double().sum(1))


@pytest.mark.parametrize("C,relu,res", [(64, True, False), (256, True, True), (2048, False, False),
                                        (24, True, True)])
def test_bn_fwd_bwd(C, relu, res):
    from mauv import ops
    G, B, H = 3, 4, 5
    M = B * H * H
    torch.manual_seed(3)
    y = torch.randn(G, M, C) * 3 + 2
    gamma, beta = torch.rand(C) + 0.5, torch.randn(C)
    rm, rv = torch.randn(C), torch.rand(C) + 0.5
    r = torch.randn(G, M, C) if res else None
    yd = y.to(dev)
    rmd, rvd = rm.clone().to(dev), rv.clone().to(dev)
    wsz = ops.bn_workspace_floats(G, M, C)
    ws = torch.empty(wsz, device=dev)
    mean, invstd, scale, shift = (torch.empty(G, C, device=dev) for _ in range(4))
    out = torch.empty(G, M, C, device=dev)
    ops.bn_fwd_train(yd, G, M, C, gamma.to(dev), beta.to(dev), rmd, rvd, 0.1, 1e-5, ws, mean,
                     invstd, scale, shift, None if r is None else r.to(dev), relu, out)
    # reference: G sequential torch BN calls in train mode
    bn = torch.nn.BatchNorm2d(C).double()
    bn.weight.data.copy_(gamma)
    bn.bias.data.copy_(beta)
    bn.running_mean.copy_(rm)
    bn.running_var.copy_(rv)
    refs, xs = [], []
    for g in range(G):
        xg = y[g].double().view(B, H, H, C).permute(0, 3, 1, 2).requires_grad_(True)
        o = bn(xg)
        if r is not None:
            o = o + r[g].double().view(B, H, H, C).permute(0, 3, 1, 2)
        if relu:
            o = torch.relu(o)
        refs.append(o)
        xs.append(xg)
    ref = torch.stack([o.permute(0, 2, 3, 1).reshape(M, C) for o in refs])
    close(out, ref)
    close(rmd, bn.running_mean)
    close(rvd, bn.running_var)
    dout = torch.randn(G, M, C)
    loss = sum((o.permute(0, 2, 3, 1).reshape(M, C) * dout[g].double()).sum()
               for g, o in enumerate(refs))
    loss.backward()
    dy = torch.empty(G, M, C, device=dev)
    dres = torch.empty(G, M, C, device=dev) if res else None
    dg = torch.zeros(C, device=dev)
    db = torch.zeros(C, device=dev)
    ops.bn_bwd(yd, out, dout.to(dev), relu, mean, invstd, scale, G, M, C, ws, dy, dres, dg, db)
    close(dy, torch.stack([x.grad.permute(0, 2, 3, 1).reshape(M, C) for x in xs]))
    close(dg, bn.weight.grad)
    close(db, bn.bias.grad)


def test_pools():
    from mauv import ops
    N, H, C = 3, 9, 64
    torch.manual_seed(4)
    x = torch.randn(N, H, H, C)
    x[0, :3, :3, :] = 0.0  # ties (post-ReLU zeros) exercise the first-max rule
    Ho = ops.out_hw(H, 3, 2, 1)
    y = torch.empty(N, Ho, Ho, C, device=dev)
    idx = torch.empty(N, Ho, Ho, C, dtype=torch.uint8, device=dev)
    ops.maxpool_fwd(x.to(dev), N, H, H, C, y, idx)
    xr = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    close(y, yr.permute(0, 2, 3, 1))
    dy = torch.randn(N, Ho, Ho, C)
    yr.backward(dy.double().permute(0, 3, 1, 2))
    dx = torch.empty(N, H, H, C, device=dev)
    ops.maxpool_bwd(dy.to(dev), idx, N, H, H, C, dx)
    close(dx, xr.grad.permute(0, 2, 3, 1))
    a = torch.empty(N, C, device=dev)
    ops.avgpool_fwd(x.to(dev), N, H * H, C, a)
    close(a, x.double().mean((1, 2)))
    da = torch.randn(N, C)
    dxa = torch.empty(N, H, H, C, device=dev)
    ops.avgpool_bwd(da.to(dev), N, H * H, C, dxa)
    close(dxa, (da.double() / (H * H))[:, None, None, :].expand(N, H, H, C))


def test_reparam_and_kl():
    from mauv import ops
    G, Cout, Cin, R = 3, 16, 8, 3
    torch.manual_seed(5)
    mu = torch.randn(Cout, Cin, R, R) * 0.1
    rho = torch.log(torch.expm1(0.1 * mu.abs()) + 1e-20)
    eps = torch.randn(G, Cout * Cin * R * R)
    out = torch.empty(G, Cout, R, R, Cin, device=dev)
    ops.reparam_sample(mu.to(dev), rho.to(dev), out, G, 0, 0, 0, Cout, Cin, R * R,
                       eps=eps.to(dev))
    sig = torch.log1p(torch.exp(rho.double()))
    ref = (mu.double() + sig * eps.double().view(G, Cout, Cin, R, R)).permute(0, 1, 3, 4, 2)
    close(out, ref)
    # backward with explicit eps
    dws = torch.randn(2, G, Cout, R, R, Cin)
    dmu = torch.zeros(Cout, Cin, R, R, device=dev)
    drho = torch.zeros_like(dmu)
    ops.reparam_bwd(dws.to(dev), 2, mu.to(dev), rho.to(dev), dmu, drho, G, 0, 0, 0, Cout, Cin,
                    R * R, eps=eps.to(dev))
    dW = dws.double().sum(0).permute(0, 1, 4, 2, 3)  # [G][Cout][Cin][R][R]
    close(dmu, dW.sum(0))
    close(drho, (dW * eps.double().view(G, Cout, Cin, R, R)).sum(0) * torch.sigmoid(rho.double()))
    # Philox path: G-batched sample == G sequential single-sample draws
    outb = torch.empty(G, Cout, R, R, Cin, device=dev)
    ops.reparam_sample(mu.to(dev), rho.to(dev), outb, G, 42, 10, 7, Cout, Cin, R * R)
    for g in range(G):
        o1 = torch.empty(1, Cout, R, R, Cin, device=dev)
        ops.reparam_sample(mu.to(dev), rho.to(dev), o1, 1, 42, 10 + g, 7, Cout, Cin, R * R)
        assert torch.equal(o1[0], outb[g])


@pytest.mark.parametrize("G,Cout,Cin,R,fixed,splits", [
    (11, 24, 20, 3, -1, 3), (11, 8, 70, 1, -1, 3), (5, 24, 20, 3, 2, 3), (12, 16, 64, 3, -1, 3),
    # 16-byte kernel (reparam_bwd4): 1x1 with a ragged 256-channel block and 1024 threads,
    # 16 quads per block in exact mode (256 threads), 3x3 with 16-channel blocks
    (5, 16, 300, 1, 2, 20), (3, 8, 64, 1, -1, 7), (5, 32, 128, 3, 4, 9), (2, 4, 12, 1, 1, 1)])
def test_reparam_bwd_sample_batches(G, Cout, Cin, R, fixed, splits):
    """reparam_bwd with more MC samples than one LDS batch (RB_GC = 8): the per-sample terms
    are added in sample order onto nonzero accumulated gradients; ragged channel blocks
    (Cin % 16, Cin % 64, Cin % 256), 1x1 and 3x3, 1 to 20 split-K slabs, both kernels (Cin % 4
    selects the 16-byte one), and bayesian-torch's fixed-sample mode."""
    from mauv import ops
    torch.manual_seed(9)
    mu = torch.randn(Cout, Cin, R, R) * 0.1
    rho = torch.randn(Cout, Cin, R, R) - 3
    eps = torch.randn(G, Cout * Cin * R * R)
    dws = torch.randn(splits, G, Cout, R, R, Cin)
    dmu0 = torch.randn(Cout, Cin, R, R)
    drho0 = torch.randn(Cout, Cin, R, R)
    dmu, drho = dmu0.clone().to(dev), drho0.clone().to(dev)
    ops.reparam_bwd(dws.to(dev), splits, mu.to(dev), rho.to(dev), dmu, drho, G, 0, 0, 0, Cout,
                    Cin, R * R, eps=eps.to(dev), fixed_sample=fixed)
    dW = dws.double().sum(0).permute(0, 1, 4, 2, 3)  # [G][Cout][Cin][R][R]
    e = eps.double().view(G, Cout, Cin, R, R)
    if fixed >= 0:
        e = e[fixed].expand_as(e)
    close(dmu, dmu0.double() + dW.sum(0))
    close(drho, drho0.double() + (dW * e).sum(0) * torch.sigmoid(rho.double()))


def test_philox_matches_oracle_restatement():
    from mauv import ops
    from oracle.philox_ref import philox4x32_10, normal4
    raw, nrm = ops.philox_raw(0x1234_5678_9ABC, 77, 3, 1000)
    ref_raw = philox4x32_10(np.arange(1000, dtype=np.uint64), 77, 3, 0x1234_5678_9ABC)
    assert np.array_equal(raw.cpu().numpy().view(np.uint32).reshape(-1, 4), ref_raw)
    np.testing.assert_allclose(nrm.cpu().numpy().reshape(-1, 4), normal4(ref_raw), atol=1e-4,
                               rtol=1e-5)
    z = nrm.cpu().double()
    assert abs(z.mean()) < 0.05 and abs(z.std() - 1) < 0.05


@pytest.mark.parametrize("hid", [128, 32, 100, 200])
def test_head_kernels(hid):
    """AdditiveAttention epilogues (base_models.py:43-52) at the model's hidden width (128)
    and at widths that are not / are more than one wave of columns."""
    from mauv import ops
    rows, H = 6, hid
    torch.manual_seed(6)
    qkv = torch.randn(rows, 3 * H)
    s = torch.randn(rows, H)
    t = torch.empty(rows, H, device=dev)
    ops.attn_t(qkv.to(dev), rows, H, t)
    close(t, torch.tanh(qkv[:, :H].double() + qkv[:, H:2 * H].double()))
    comb = torch.zeros(rows, 3 * H, device=dev)
    ops.attn_out(qkv.to(dev), s.to(dev), rows, H, comb, 3 * H, H)
    sr = s.double().requires_grad_(True)
    vr = qkv[:, 2 * H:].double().requires_grad_(True)
    o = vr * torch.softmax(sr, 1)
    close(comb[:, H:2 * H], o)
    do = torch.randn(rows, H)
    o.backward(do.double())
    dcomb = torch.zeros(rows, 3 * H)
    dcomb[:, H:2 * H] = do
    dqkv = torch.zeros(rows, 3 * H, device=dev)
    ds = torch.empty(rows, H, device=dev)
    ops.attn_out_bwd(dcomb.to(dev), 3 * H, H, qkv.to(dev), s.to(dev), rows, H, dqkv, ds)
    close(ds, sr.grad)
    close(dqkv[:, 2 * H:], vr.grad)
    dt = torch.randn(rows, H)
    ops.attn_t_bwd(dt.to(dev), t, rows, H, dqkv)
    tt = torch.tanh(qkv[:, :H].double() + qkv[:, H:2 * H].double())
    close(dqkv[:, :H], dt.double() * (1 - tt * tt))
    close(dqkv[:, H:2 * H], dt.double() * (1 - tt * tt))


def test_mc_head_kernels():
    from mauv import ops
    G, B, C = 5, 9, 7
    torch.manual_seed(7)
    logits = torch.randn(G, B, C)
    labels = torch.randint(0, C, (B,))
    mean = torch.empty(B, C, device=dev)
    loss = torch.empty(1, device=dev)
    ops.mc_mean_ce(logits.to(dev), labels.to(dev), G, B, C, mean, loss)
    lr = logits.double().requires_grad_(True)
    m = lr.mean(0)
    ce = F.cross_entropy(m, labels)
    close(mean, m)
    close(loss, ce.reshape(1))
    ce.backward()
    dl = torch.empty(G, B, C, device=dev)
    g = torch.tensor([1.0], device=dev)
    ops.mc_mean_bwd(None, g, mean, labels.to(dev), G, B, C, dl)
    close(dl, lr.grad)
    sums = torch.empty(B, 2 * C + 1, dtype=torch.float64, device=dev)
    ops.mc_stats(logits.to(dev), G, B, C, 1e-7, sums)
    mp = torch.empty(B, C, device=dev)
    var = torch.empty(B, device=dev)
    alea = torch.empty(B, device=dev)
    pe = torch.empty(B, device=dev)
    pred = torch.empty(B, dtype=torch.int64, device=dev)
    ops.mc_finalize(sums, G, B, C, 1e-8, mp, var, alea, pe, pred)
    P = torch.softmax(logits.double(), -1)
    close(mp, P.mean(0))
    close(var, torch.var(P, 0).mean(1))
    close(alea, torch.mean(-torch.sum(P * torch.log(P + 1e-7), -1), 0))
    close(pe, -torch.sum(P.mean(0) * torch.log(P.mean(0) + 1e-8), 1))
    assert torch.equal(pred.cpu(), torch.argmax(P.mean(0), 1))
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    x = torch.randn(10000, device=dev)
    ops.nonfinite_count(x, cnt)
    assert cnt.item() == 0
    x[777] = float("nan")
    ops.nonfinite_count(x, cnt)
    assert cnt.item() > 0


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
def test_bn_apply_pending_residual_bn(dt):
    """bn3 apply with the downsample BN folded in: relu(y*s+h + r*rs+rh)."""
    from mauv import ops
    G, M, C = 2, 50, 256
    torch.manual_seed(9)
    y, r = (torch.randn(G, M, C).to(dt).to(dev) for _ in range(2))
    s, h, rs, rh = (torch.randn(G, C, device=dev) for _ in range(4))
    out = torch.empty(G, M, C, device=dev, dtype=dt)
    ops.bn_apply(y, s, h, r, True, out, G, M, C, res_bn=(rs, rh))
    ref = torch.relu(y.float() * s[:, None] + h[:, None] + r.float() * rs[:, None] + rh[:, None])
    tol = 1e-5 if dt == torch.float32 else 2 ** -7
    close(out.float(), ref, rtol=tol, atol=tol)


def test_fused_adam_matches_torch_adam():
    """mauv.optim.FusedAdam == torch.optim.Adam (weight decay on, 3 steps, several tensors
    incl. a numel % 4 tail); state_dict interchangeable."""
    from mauv.optim import FusedAdam
    torch.manual_seed(11)
    shapes = [(64, 3, 7, 7), (7,), (1284, 384), (5, 3)]
    pa = [torch.randn(s, device=dev, requires_grad=True) for s in shapes]
    pb = [p.detach().clone().requires_grad_(True) for p in pa]
    oa = FusedAdam(pa, lr=5e-3, weight_decay=1e-5)
    ob = torch.optim.Adam(pb, lr=5e-3, weight_decay=1e-5)
    for _ in range(3):
        gs = [torch.randn(s, device=dev) for s in shapes]
        for p, q, g in zip(pa, pb, gs):
            p.grad, q.grad = g.clone(), g.clone()
        oa.step()
        ob.step()
    for p, q in zip(pa, pb):
        close(p, q, rtol=1e-6, atol=1e-7)
    ob2 = torch.optim.Adam(pb, lr=5e-3, weight_decay=1e-5)
    ob2.load_state_dict(oa.state_dict())
    for p, q in zip(pa, pb):
        close(ob2.state[q]["exp_avg_sq"], oa.state[p]["exp_avg_sq"], rtol=1e-6, atol=1e-12)


def test_fused_adam_fast_path_matches_torch_adam():
    """Persistent gradient tensors (the engine's arena views): from the second step FusedAdam
    takes its cached path (one table, one shared step buffer) — still == torch.optim.Adam over 5
    steps, state["step"] readable per parameter, and a state_dict round trip (torch Adam ->
    FusedAdam) continues identically."""
    from mauv.optim import FusedAdam
    torch.manual_seed(12)
    shapes = [(64, 3, 7, 7), (7,), (300, 20), (5, 3)]
    pa = [torch.randn(s, device=dev, requires_grad=True) for s in shapes]
    pb = [p.detach().clone().requires_grad_(True) for p in pa]
    for p, q in zip(pa, pb):
        p.grad, q.grad = torch.empty_like(p), torch.empty_like(q)
    oa = FusedAdam(pa, lr=5e-3, weight_decay=1e-5)
    ob = torch.optim.Adam(pb, lr=5e-3, weight_decay=1e-5)
    for _ in range(5):
        for p, q in zip(pa, pb):
            g = torch.randn_like(p)
            p.grad.copy_(g)
            q.grad.copy_(g)
        oa.step()
        ob.step()
    assert 0 in oa._fast and all(float(oa.state[p]["step"]) == 5.0 for p in pa)
    for p, q in zip(pa, pb):
        close(p, q, rtol=1e-6, atol=1e-7)
    import copy
    oa2 = FusedAdam(pa, lr=5e-3, weight_decay=1e-5)
    # a copy: torch's load_state_dict keeps the very "step" tensors it is given (no copy), so
    # two optimizers loaded from one dict would bump each other's counts
    oa2.load_state_dict(copy.deepcopy(ob.state_dict()))
    for p, q in zip(pa, pb):
        g = torch.randn_like(p)
        p.grad.copy_(g)
        q.grad.copy_(g)
    oa2.step()
    ob.step()
    for p, q in zip(pa, pb):
        close(p, q, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("nblk", [37, 1500])
def test_bn_stats_finalize_segmented(nblk):
    """Per-128-row partials (count, mean, M2) merged into batch statistics: one launch up to
    512 partials per channel, segmented two-stage Chan merge beyond (MC-batched inference
    chunks reach tens of thousands) — vs float64 statistics of the full data."""
    from mauv import ops
    G, C, rows = 2, 64, 128
    torch.manual_seed(4)
    M = nblk * rows - 57                                   # ragged last partial
    y = torch.randn(G, M, C, dtype=torch.float64) * 3 + torch.linspace(-5, 5, C, dtype=torch.float64)
    cnt = torch.full((nblk,), float(rows), dtype=torch.float64)
    cnt[-1] = rows - 57
    pm = torch.empty(G, nblk, C, dtype=torch.float64)
    p2 = torch.empty(G, nblk, C, dtype=torch.float64)
    for b in range(nblk):
        blk = y[:, b * rows:min(M, (b + 1) * rows)]
        pm[:, b] = blk.mean(1)
        p2[:, b] = ((blk - blk.mean(1, keepdim=True)) ** 2).sum(1)
    gamma, beta = torch.rand(C) + 0.5, torch.randn(C)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    ws = torch.empty(ops.bn_stats_workspace_floats(G, nblk, C), device=dev)
    st = torch.empty(4, G, C, device=dev)
    ops.bn_stats_finalize(G, nblk, C, pm.float().to(dev), p2.float().to(dev),
                          cnt.float().expand(G, nblk).contiguous().to(dev), gamma.to(dev),
                          beta.to(dev), rm, rv, 0.1, 1e-5, ws, st[0], st[1], st[2], st[3])
    mean, var = y.mean(1), y.var(1, unbiased=False)
    close(st[0], mean, rtol=1e-6, atol=1e-6)
    close(st[1], 1.0 / torch.sqrt(var + 1e-5), rtol=1e-6, atol=0)
    uvar = y.var(1, unbiased=True)
    ref_rv = torch.ones(C, dtype=torch.float64)
    for g in range(G):
        ref_rv = 0.9 * ref_rv + 0.1 * uvar[g]
    close(rv, ref_rv, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("C,M", [(24, 1000), (512, 1000), (2056, 37), (64, 3000)])
def test_bn_apply_row_walk_ragged(C, M):
    """Row-walk apply (C <= 2048; 256/(C/8) rows in parallel, 8 rows a thread) over ragged
    row counts and a non-power-of-two C; C > 2048 takes the grid-stride form."""
    from mauv import ops
    G = 3
    torch.manual_seed(11)
    y = torch.randn(G, M, C, device=dev)
    r = torch.randn(G, M, C, device=dev)
    s, h = torch.randn(G, C, device=dev), torch.randn(G, C, device=dev)
    out = torch.full((G, M, C), float("nan"), device=dev)
    ops.bn_apply(y, s, h, r, True, out, G, M, C)
    ref = torch.relu(y.double() * s.double()[:, None] + h.double()[:, None] + r.double())
    assert torch.allclose(out.double(), ref, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16],
                         ids=["fp32", "bf16", "f16"])
def test_maxpool_bn_fused_matches_materialised(dt):
    """Stem bn1 + ReLU applied inside the max-pool == bn_apply then max-pool, bit for bit
    (pooled values and argmax bytes), per MC group; idx=None skips the argmax."""
    from mauv import ops
    G, B, H, W, C = 2, 3, 17, 15, 64
    N = G * B
    torch.manual_seed(21)
    y = (torch.randn(G, B, H, W, C, device=dev) * 2).to(dt)
    s, h = torch.randn(G, C, device=dev), torch.randn(G, C, device=dev)
    s[:, :8] = 0.0            # ties: whole windows of zeros after the ReLU
    y[0, 1, 4, 5, 8:20] = float("nan")   # NaN taps: relu(NaN * s + h) stores 0 in every path
    a = torch.empty_like(y)
    ops.bn_apply(y, s, h, None, True, a, G, B * H * W, C)
    Ho, Wo = ops.out_hw(H, 3, 2, 1), ops.out_hw(W, 3, 2, 1)
    p_ref = torch.empty(G, B, Ho, Wo, C, device=dev, dtype=dt)
    i_ref = torch.empty(G, B, Ho, Wo, C, device=dev, dtype=torch.uint8)
    ops.maxpool_fwd(a, N, H, W, C, p_ref, i_ref)
    p = torch.full_like(p_ref, float("nan"))
    i = torch.full_like(i_ref, 255)
    ops.maxpool_fwd(y, N, H, W, C, p, i, bn=(s, h, G))
    assert torch.equal(p.view(torch.int16 if dt != torch.float32 else torch.int32),
                       p_ref.view(torch.int16 if dt != torch.float32 else torch.int32))
    assert torch.equal(i, i_ref)
    p2 = torch.full_like(p_ref, float("nan"))
    ops.maxpool_fwd(y, N, H, W, C, p2, None, bn=(s, h, G))
    assert torch.equal(p2, p_ref)
    ref = F.max_pool2d(a.float().reshape(N, H, W, C).permute(0, 3, 1, 2), 3, 2, 1)
    assert torch.equal(p_ref.float().reshape(N, Ho, Wo, C).permute(0, 3, 1, 2), ref)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
@pytest.mark.parametrize("C,M,res_bn", [(256, 300, False), (2048, 37, True), (24, 1000, False)])
def test_bn_relu_mask_path_matches_output_path(dt, C, M, res_bn):
    """bn_apply_mask / bn_bwd_mask (1-bit ReLU masks) == bn_apply / bn_bwd reading the stored
    output, bit for bit: out, dy, dres, dgamma, dbeta."""
    from mauv import ops
    G = 3
    torch.manual_seed(23)
    y = (torch.randn(G, M, C, device=dev) * 2).to(dt)
    r = torch.randn(G, M, C, device=dev).to(dt)
    s, h = torch.randn(G, C, device=dev), torch.randn(G, C, device=dev)
    s[:, :8] = 0.0          # outputs exactly 0 -> masked
    rb = (torch.randn(G, C, device=dev), torch.randn(G, C, device=dev)) if res_bn else None
    out_ref = torch.empty_like(y)
    ops.bn_apply(y, s, h, r, True, out_ref, G, M, C, res_bn=rb)
    out = torch.full_like(y, float("nan"))
    mask = torch.empty(G * M * C // 8, dtype=torch.uint8, device=dev)
    ops.bn_apply_mask(y, s, h, r, out, mask, G, M, C, res_bn=rb)
    assert torch.equal(out, out_ref)
    bits = ((mask.view(-1, 1).int() >> torch.arange(8, device=dev)) & 1).view(G, M, C)
    assert torch.equal(bits.bool(), out_ref.float() > 0)
    mean, invstd = torch.randn(G, C, device=dev), torch.rand(G, C, device=dev) + 0.5
    dout = torch.randn(G, M, C, device=dev).to(dt)
    res = []
    for use_mask in (False, True):
        ws = torch.empty(ops.bn_workspace_floats(G, M, C), device=dev)
        dy, dres = torch.empty_like(y), torch.empty_like(y)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        if use_mask:
            ops.bn_bwd_mask(y, mask, dout, mean, invstd, s, G, M, C, ws, dy, dres, dg, db)
        else:
            ops.bn_bwd(y, out_ref, dout, True, mean, invstd, s, G, M, C, ws, dy, dres, dg, db,
                       shift=h)
        res.append((dy, dres, dg, db))
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16],
                         ids=["fp32", "bf16", "f16"])
@pytest.mark.parametrize("G,Cout,Cin,R,cin_pad,explicit", [
    (5, 64, 64, 3, None, False), (5, 48, 1028, 1, None, False), (3, 7, 2048, 1, None, True),
    (4, 33, 20, 3, 24, True), (2, 16, 12, 7, None, False), (5, 8, 6, 3, None, False)])
def test_reparam_sample_block_form_bit_identical(dt, G, Cout, Cin, R, cin_pad, explicit):
    """The block-form sampling (one output channel x channel range per block, LDS image, vector
    KRSC stores; mauv_set_reparam_kernels bit 0) writes the per-element kernel's values: Philox
    and explicit eps, 1x1 / 3x3 / 7x7, ragged channel ranges (1028 = 1024 + 4), padded KRSC rows
    (pad channels untouched), the device sample counter; Cin % 4 != 0 falls back.  Its 16-bit
    weights are the fp32 sample rounded once more (the reference's fp32 weight cast by autocast)
    — bit-exact for every dtype; the per-element f16 kernel instead rounds mu + sigma*eps to f16
    in one step (hipcc contracts it to v_fma_mix), which differs by 1 ulp on rare elements."""
    from mauv import ops
    torch.manual_seed(21)
    RS = R * R
    mu = (torch.randn(Cout, Cin, R, R) * 0.1).to(dev)
    rho = (torch.randn(Cout, Cin, R, R) - 3).to(dev)
    eps = torch.randn(G, Cout * Cin * RS, device=dev) if explicit else None
    cp = cin_pad or Cin
    base = torch.tensor([3], dtype=torch.int64, device=dev)
    outs = []
    prev = ops.set_reparam_kernels(sample_blk=False)
    try:
        for blk in (False, True):
            ops.set_reparam_kernels(sample_blk=blk)
            o = torch.full((G, Cout, R, R, cp), 7.0, device=dev).to(dt)
            ops.reparam_sample(mu, rho, o, G, 99, 11, 5, Cout, Cin, RS, eps=eps,
                               cin_pad=cin_pad)
            o2 = torch.full((G, Cout, R, R, cp), 7.0, device=dev).to(dt)
            ops.reparam_sample_ex(mu, rho, o2, G, 99, 11, base, 5, Cout, Cin, RS, eps=eps,
                                  cin_pad=cin_pad)
            outs.append((o, o2))
    finally:
        ops.set_reparam_kernels(sample_blk=prev[0])
    f32 = torch.full((G, Cout, R, R, cp), 7.0, device=dev)
    ops.reparam_sample(mu, rho, f32, G, 99, 11, 5, Cout, Cin, RS, eps=eps, cin_pad=cin_pad)
    torch.cuda.synchronize()
    blk_on = Cin % 4 == 0
    if blk_on or dt != torch.float16:
        assert torch.equal(outs[1][0], f32.to(dt))
    if dt == torch.float16:
        for a, b in ((outs[0][0], outs[1][0]), (outs[0][1], outs[1][1])):
            d = (a.view(torch.int16).int() - b.view(torch.int16).int()).abs()
            assert d.max() <= 1 and (d > 0).float().mean() < 1e-3
    else:
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    if cin_pad:
        assert (outs[1][0][..., Cin:].float() == 7.0).all()
    if not explicit:   # the device counter shifts the sample index by 3
        assert not torch.equal(outs[1][0], outs[1][1])


@pytest.mark.parametrize("Cin,Cout,R,st,H,form", [
    (256, 64, 1, 1, 16, "masked"),      # K = 64: the short-K (SEQ) kernel, half-tile LDS passes
    (256, 512, 1, 1, 15, "masked"),     # pipelined 128 x 128 tiles, ragged M
    (128, 128, 3, 1, 9, "addend"),      # 3x3, addend without mask bits
    (256, 512, 1, 2, 16, "accumulate"), # stride-2 downsample class accumulating into dx
    (192, 256, 3, 2, 11, "both"),       # strided 3x3, ragged classes, addend + accumulate
    (96, 64, 1, 1, 7, "masked"),        # 64-wide tiles (64 x 64 kernel)
])
def test_dgrad_f32_staged_epilogue(Cin, Cout, R, st, H, form):
    """fp32 data gradients with a residual addend (under ReLU-mask bits or not) and / or
    accumulation into dx: the LDS-staged 16-byte epilogue (conv_common.h staged_epilogue_f32)
    against float64 — the addend counted exactly where the mask bit is set, classes without taps
    leaving dx (+ addend) as it was."""
    from mauv import ops
    G, B = 2, 2
    pd = R // 2
    torch.manual_seed(8)
    Ho = ops.out_hw(H, R, st, pd)
    dy = torch.randn(G, B, Ho, Ho, Cout)
    w = torch.randn(G, Cout, R, R, Cin) / (Cout * R * R) ** 0.5
    ad = torch.randn(G, B, H, H, Cin) if form in ("masked", "addend", "both") else None
    mask = None
    keep = torch.ones(G, B, H, H, Cin, dtype=torch.bool)
    if form == "masked":
        keep = torch.rand(G, B, H, H, Cin) > 0.4
        bits = keep.reshape(-1, 8).to(torch.uint8) << torch.arange(8, dtype=torch.uint8)
        mask = bits.sum(1).to(torch.uint8).to(dev)
    dx0 = torch.randn(G, B, H, H, Cin)
    acc = form in ("accumulate", "both")
    dx = dx0.clone().to(dev) if acc else torch.full((G, B, H, H, Cin), float("nan"), device=dev)
    ops.conv2d_bwd_data(dy.to(dev), w.to(dev), dx, G, B, H, H, Cin, Cout, R, st, pd,
                        addend=None if ad is None else ad.to(dev), accumulate=acc,
                        addend_mask=mask)
    ref = []
    for g in range(G):
        xg = torch.zeros(B, Cin, H, H, dtype=torch.float64, requires_grad=True)
        F.conv2d(xg, w[g].permute(0, 3, 1, 2).double(), stride=st, padding=pd).backward(
            dy[g].permute(0, 3, 1, 2).double())
        ref.append(xg.grad.permute(0, 2, 3, 1))
    ref = torch.stack(ref)
    if ad is not None:
        ref = ref + torch.where(keep, ad.double(), torch.zeros((), dtype=torch.float64))
    if acc:
        ref = ref + dx0.double()
    assert not torch.isnan(dx).any()
    close(dx, ref, rtol=1e-5, atol=1e-5)
