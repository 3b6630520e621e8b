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
def test_conv16_lazy_bn_input_and_stats(dt):
    """x' = relu(x*scale + shift) applied on load (FWD and WGRAD) + epilogue statistics."""
    from mauv import ops
    G, B, H, Cin, Cout = 2, 3, 8, 64, 128
    torch.manual_seed(3)
    x = torch.randn(G, B, H, H, Cin).to(dt)
    sc = torch.rand(G, Cin) + 0.5
    sh = torch.randn(G, Cin) * 0.3
    w = (torch.randn(G, Cout, 3, 3, Cin) / 24).to(dt)
    xt = torch.relu(x.float() * sc[:, None, None, None] + sh[:, None, None, None]).to(dt)
    ref = ref_conv(xt, w, 1, 1)
    nblk = ops.fwd_stat_blocks(G, B, H, H, Cin, Cout, 3, 1, 1)
    pm = torch.empty(G, nblk, Cout, device=dev)
    pm2 = torch.empty_like(pm)
    pc = torch.empty(G, nblk, device=dev)
    y = torch.empty(G, B, H, H, Cout, device=dev, dtype=dt)
    ops.conv2d_fwd(x.to(dev), w.to(dev), y, G, B, H, H, Cin, Cout, 3, 1, 1,
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
    splits = ops.wgrad_splits(G, B, H, H, Cin, Cout, 3, 1, 1)
    ws = torch.empty(splits, G, Cout, 9 * Cin, device=dev)
    ops.conv2d_bwd_weight(x.to(dev), dy.to(dev), ws, splits, G, B, H, H, Cin, Cout, 3, 1, 1,
                          x_bn=(sc.to(dev), sh.to(dev), 1))
    dw = []
    for g in range(G):
        wg = w[g].permute(0, 3, 1, 2).double().requires_grad_(True)
        F.conv2d(xt[g].permute(0, 3, 1, 2).double(), wg, padding=1).backward(
            dy[g].permute(0, 3, 1, 2).double())
        dw.append(wg.grad.permute(0, 2, 3, 1))
    close(ws.sum(0).view(G, Cout, 3, 3, Cin), torch.stack(dw), 1e-3)
