"""Thin tensor-level wrappers over the libmauv_hip C-ABI (include/mauv.h).

Every function launches on the current torch stream and is asynchronous; tensors must be
contiguous device tensors of the documented dtype.  These wrappers do no arithmetic of
their own — all compute is in the HIP kernels.
"""
import ctypes

import torch

from ._lib import lib, check, MauvRoute

_LL5 = ctypes.c_longlong * 5


def _p(t):
    return None if t is None else t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


H16 = {torch.bfloat16: 0, torch.float16: 1}   # C-ABI dtype codes of the 16-bit path


def _raise(t, dt):
    cur = torch.cuda.current_device() if t.is_cuda else None
    raise ValueError(f"mauv kernel operand must be a contiguous {dt} tensor on the current ROCm "
                     f"device cuda:{cur} (the launch stream's), got {t.dtype} on {t.device} "
                     f"(contiguous={t.is_contiguous()}, shape={tuple(t.shape)})")


def _h16(dt, *ts):
    cur = None
    for t in ts:
        if t is None:
            continue
        if not (t.is_cuda and t.dtype == dt and t.is_contiguous()):
            _raise(t, dt)
        if cur is None:
            cur = torch.cuda.current_device()
        if t.device.index != cur:
            _raise(t, dt)


def _f32(*ts):
    _h16(torch.float32, *ts)


def _dev(dt, *ts):
    """Every tensor handed to a kernel is a contiguous device tensor of dtype ``dt`` on the
    device whose current stream the launch uses: a host pointer (or another GPU's) reaching a
    HIP kernel is a memory-access fault the caller cannot catch."""
    _h16(dt, *ts)


def out_hw(H, R, stride, pad):
    return (H + 2 * pad - R) // stride + 1


# ----------------------------------------------------------------------- profiling hook
# bench.py sets PROFILE to a list to time every implicit-GEMM launch with HIP events on the
# stream the kernel runs on (torch's current stream); entries: (kind, flops, bytes, launches,
# ev0, ev1) — a strided dgrad call is stride^2 kernel launches (one per output-parity class)
# with the ALGORITHMIC bytes of the launch (every operand read once, every output written once).
PROFILE_INFO = None   # when a list (with PROFILE): one shape tuple per PROFILE row
PROFILE = None


class _Prof:
    __slots__ = ("kind", "flops", "nbytes", "launches", "e0", "info")

    def __init__(self, kind, flops, nbytes=0.0, launches=1, info=None):
        self.kind, self.flops, self.nbytes, self.launches = kind, flops, nbytes, launches
        self.info = info

    def __enter__(self):
        if PROFILE is not None:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e0.record()

    def __exit__(self, *a):
        if PROFILE is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            PROFILE.append((self.kind, self.flops, self.nbytes, self.launches, self.e0, e1))
            if PROFILE_INFO is not None:   # the launch's shape, parallel to PROFILE (tools/)
                PROFILE_INFO.append(self.info)


# ----------------------------------------------------------------------- convolutions
F32_MATH = {"exact": 0, "split3": 3, "split1": 5, "split": 6}
_F32_NAMES = {v: k for k, v in F32_MATH.items()}


def route():
    """The library's kernel routing (include/mauv.h MauvRoute) as a dict of its fields."""
    r = MauvRoute()
    check(lib.mauv_get_route(ctypes.byref(r)), "get_route")
    return {f: getattr(r, f) for f, _ in MauvRoute._fields_ if f != "reserved"}


def set_route(**fields):
    """Change the named MauvRoute fields (process-wide; between launches only, include/mauv.h);
    returns the previous values of those fields."""
    r = MauvRoute()
    check(lib.mauv_get_route(ctypes.byref(r)), "get_route")
    prev = {}
    for k, v in fields.items():
        if k == "reserved" or not hasattr(r, k):
            raise ValueError(f"MauvRoute has no field {k!r}")
        prev[k] = getattr(r, k)
        setattr(r, k, int(v))
    check(lib.mauv_set_route(ctypes.byref(r)), "set_route")
    return prev


def f32_math():
    """Arithmetic of the fp32 convs: "split" (default; exact three-way bf16 split of every
    operand, six plane products on bf16 MFMA, fp32 accumulation), "split1", "split3" or "exact"
    (v_mfma_f32_32x32x2_f32) — include/mauv.h MauvRoute.f32_math."""
    return _F32_NAMES[route()["f32_math"]]


def set_f32_math(mode):
    """Select the fp32 conv arithmetic (process-wide); returns the previous mode."""
    return _F32_NAMES[set_route(f32_math=F32_MATH[mode])["f32_math"]]


def _mode(mode, key):
    """None: keep; True / False: 2 / 0 (big16, expand16) or 1 / 0; else the int."""
    if mode is None:
        return route()[key]
    if mode is True:
        return 2 if key in ("big16", "expand16") else 1
    return 0 if mode is False else int(mode)


def set_halo3(on):
    """Route the 16-bit 3x3 / stride-1 64 -> 64 convs through the LDS-row-image kernel
    (True, default) or the implicit GEMM (False); returns the previous setting."""
    return bool(set_route(halo3=1 if on else 0)["halo3"])


def set_big16(mode=None, min_k=0):
    """Route 16-bit forwards through the 256-row LDS-DMA kernel: 1 (default) where it measured
    faster, 2 (or True) every forward it covers with K >= min_k, 0 (or False) none; None /
    min_k=0 keep.  Returns the previous mode (0 / 1 / 2)."""
    f = {"big16": _mode(mode, "big16")}
    if min_k > 0:
        f["big16_min_k"] = int(min_k)
    return set_route(**f)["big16"]


def set_expand16(mode=None):
    """Route 16-bit 1x1 / stride-1 expansion forwards (K = 64 / 128 / 256) through the
    weight-stationary kernel (conv_expand16.hip): 1 (default) where it measured faster, 2 (or
    True) every shape it covers, 3 as 2 with 32-column waves at K = 128, 0 (or False) none (the
    implicit GEMM), None keep.  Returns the previous mode."""
    return set_route(expand16=_mode(mode, "expand16"))["expand16"]


def set_haloc16(mode=None):
    """Route 16-bit 3x3 / stride-1 forwards over 128-512 channels through the chunked LDS
    row-image kernel (conv_haloc16.hip), and the stride-1 data gradients of the same shapes:
    1 / True (default, 32 x 64 wave tiles), 2 (64 x 64 wave tiles), 3 (the forwards only),
    0 / False (the implicit GEMM), None keep.  Returns the previous mode."""
    return set_route(haloc16=_mode(mode, "haloc16"))["haloc16"]


def set_reparam_kernels(sample_blk=None, bwd4=None):
    """Kernel forms of reparam_sample (block form, bit-identical) and reparam_bwd (16-byte slab
    loads); None keeps a setting.  Returns the previous (sample_blk, bwd4)."""
    prev = route()["reparam_kernels"]
    sb = (prev & 1) if sample_blk is None else int(bool(sample_blk))
    b4 = (prev >> 1) & 1 if bwd4 is None else int(bool(bwd4))
    set_route(reparam_kernels=sb | (b4 << 1))
    return bool(prev & 1), bool(prev & 2)


def conv2d_fwd(x, w, y, G, B, H, W, Cin, Cout, R, stride, pad, bias=None, x_strides=None,
               x_bn=None, stats=None, alg_cin=None, ysh=None):
    """y[G][B*Ho*Wo][Cout] = conv(x'[g], w[g]) (+ bias[g]); w: [G][Cout][R][R][Cin].
    x_bn = (scale [G][Cin], shift [G][Cin], relu): x' = [relu](x*scale + shift) on load.
    stats = (mean, m2, cnt) partial buffers for the epilogue BN statistics (see
    fwd_stat_blocks).  ysh ([Cout] fp32, 16-bit only): y is stored centred, y - ysh, and the
    statistics partials are those of the stored values (the accumulators start at -ysh; the
    consuming BN's centre, bn_stats_finalize takes the same ysh)."""
    xs = None if x_strides is None else _LL5(*x_strides)
    sc, sh, rl = x_bn if x_bn is not None else (None, None, 0)
    sm, s2, sn = stats if stats is not None else (None, None, None)
    Ho, Wo = out_hw(H, R, stride, pad), out_hw(W, R, stride, pad)
    xg = 1 if (x_strides is not None and x_strides[0] == 0) else G
    # profiling counts ALGORITHMIC work: a zero-padded stem input (16-bit path) counts its
    # real channels (alg_cin)
    fl = 2.0 * G * B * Ho * Wo * Cout * R * R * (alg_cin or Cin)
    esz = w.element_size()
    nb = esz * (xg * B * H * W * Cin + G * Cout * R * R * Cin + G * B * Ho * Wo * Cout)
    if ysh is not None and w.dtype not in H16:
        raise ValueError("conv2d_fwd: ysh (centred storage) is for the 16-bit convs")
    if w.dtype in H16:
        assert bias is None, "16-bit convs carry no bias (the trunks' convs are bias=False)"
        _h16(w.dtype, w, y)
        _f32(ysh)
        if ysh is not None and ysh.numel() != Cout:
            raise ValueError("conv2d_fwd: ysh needs Cout values")
        assert x.is_cuda and x.dtype == w.dtype and x.device.index == torch.cuda.current_device()
        with _Prof("fwd_" + str(w.dtype)[6:], fl, nb,
                   info=(G, B, H, W, Cin, Cout, R, stride, pad, x_bn is not None)):
            check(lib.mauv_conv2d_fwd_h16(H16[w.dtype], _p(x), xs, _p(sc), _p(sh), int(rl), _p(w),
                                          _p(y), G, B, H, W, Cin, Cout, R, R, stride, pad,
                                          _p(sm), _p(s2), _p(sn), _p(ysh), stream()),
                  "conv2d_fwd_h16")
        return
    _f32(w, y, bias)
    assert x.is_cuda and x.dtype == torch.float32 and x.device.index == torch.cuda.current_device()
    with _Prof("fwd", fl, nb, info=(G, B, H, W, Cin, Cout, R, stride, pad, x_bn is not None)):
        check(lib.mauv_conv2d_fwd_f32(_p(x), xs, _p(sc), _p(sh), int(rl), _p(w), _p(bias), _p(y),
                                      G, B, H, W, Cin, Cout, R, R, stride, pad, _p(sm), _p(s2),
                                      _p(sn), stream()), "conv2d_fwd")


def conv2d_fwd_fold(y, scale, shift, res, res_bn, out, w, y1, G, B, H, W, Cin, Cout,
                    stats=None, mask=None, ysh=None):
    """A bottleneck's 1x1 conv1 over the previous block's output formed on load
    (mauv_conv2d_fwd_fold_h16): out = relu(y*scale + shift + res'), res' = res or
    res*res_scale + res_shift (res_bn), is written through exactly as bn_apply would write it
    (mask: also its ReLU bits as bn_apply_mask writes them) and y1 = conv1x1(out) exactly as
    conv2d_fwd would compute it (ysh: y1 stored centred, as conv2d_fwd's).  True: done; False: the shape is outside the kernel and nothing
    ran (the caller runs bn_apply[_mask], then conv2d_fwd)."""
    rs, rh = res_bn if res_bn is not None else (None, None)
    if w.dtype not in H16:
        raise ValueError("conv2d_fwd_fold: 16-bit trunks only")
    _h16(w.dtype, y, res, out, w, y1)
    _f32(scale, shift, rs, rh, ysh)
    if mask is not None:
        _dev(torch.uint8, mask)
        if mask.numel() * 8 != out.numel():
            raise ValueError("conv2d_fwd_fold: mask needs out.numel() / 8 bytes")
    sm, s2, sn = stats if stats is not None else (None, None, None)
    M = B * H * W
    fl = 2.0 * G * M * Cout * Cin
    nb = w.element_size() * (3 * G * M * Cin + G * Cout * Cin + G * M * Cout)
    # its own profile kind: the launch also carries the block output's BN pass (bench.py's
    # breakdown lists it beside fwd / wgrad / dgrad)
    with _Prof("fold_" + str(w.dtype)[6:], fl, nb, info=(G, B, H, W, Cin, Cout, 1, 1, 0, True)):
        rc = lib.mauv_conv2d_fwd_fold_h16(H16[w.dtype], _p(y), _p(scale), _p(shift), _p(res),
                                          _p(rs), _p(rh), _p(out), _p(mask), _p(w), _p(y1), G, B,
                                          H, W, Cin, Cout, _p(sm), _p(s2), _p(sn), _p(ysh),
                                          stream())
    if rc == 1:
        if PROFILE is not None:
            PROFILE.pop()
        return False
    check(rc, "conv2d_fwd_fold_h16")
    return True


def fwd_stat_blocks(G, B, H, W, Cin, Cout, R, stride, pad):
    return lib.mauv_conv2d_fwd_stat_blocks(G, B, H, W, Cin, Cout, R, R, stride, pad)


def dgrad_stat_blocks(G, B, H, W, Cin, Cout, R, stride, pad):
    return lib.mauv_conv2d_bwd_data_stat_blocks(G, B, H, W, Cin, Cout, R, R, stride, pad)


def conv2d_bwd_data(dy, w, dx, G, B, H, W, Cin, Cout, R, stride, pad, addend=None,
                    accumulate=False, bn=None, addend_mask=None):
    """bn = dict(y, out|None, mask|None, scale, shift, mean, invstd, relu, p1, p2): dx is the
    output gradient of that BatchNorm; the epilogue writes its backward partial sums into p1/p2.
    addend_mask (uint8 ReLU-mask bits of dx's shape, bn_apply_mask): the addend counts only
    where the bit is set (a block output's residual gradient without a dres tensor)."""
    if addend_mask is not None:
        _dev(torch.uint8, addend_mask)
        if addend is None or addend_mask.numel() * 8 != dx.numel():
            raise ValueError("conv2d_bwd_data: addend_mask needs an addend and dx.numel()/8 bytes")
    Ho, Wo = out_hw(H, R, stride, pad), out_hw(W, R, stride, pad)
    b = bn or {}
    fl = 2.0 * G * B * Ho * Wo * Cout * R * R * Cin
    nb = w.element_size() * (G * B * Ho * Wo * Cout + G * Cout * R * R * Cin +
                             G * B * H * W * Cin * (1 + (addend is not None) + bool(accumulate)))
    # kernel launches: one per output-parity class with pixels, except the tapless classes of an
    # accumulating call without addend or partials (they add nothing and are not launched:
    # the stride-2 1x1 downsample's 3 of 4, conv_gemm.hip / conv_gemm16.hip)
    skip_tapless = bool(accumulate) and addend is None and bn is None

    def taps(p):
        r0 = (p + pad) % stride
        return (R - r0 + stride - 1) // stride if r0 < R else 0
    nl = sum(1 for ph in range(stride) for pw in range(stride)
             if (H - ph + stride - 1) // stride > 0 and (W - pw + stride - 1) // stride > 0
             and not (skip_tapless and taps(ph) * taps(pw) == 0))
    if w.dtype in H16:
        _h16(w.dtype, dy, w, dx, addend, b.get("y"), b.get("out"))
        _f32(b.get("scale"), b.get("shift"), b.get("mean"), b.get("invstd"), b.get("p1"),
             b.get("p2"))
        mk = b.get("mask")
        if mk is not None:
            _dev(torch.uint8, mk)
        if bn is not None:      # + reads y (and out / mask bits) beside each dx chunk
            nb += w.element_size() * G * B * H * W * Cin * (1 + (b.get("out") is not None))
        with _Prof("dgrad_" + str(w.dtype)[6:], fl, nb, nl,
                   info=(G, B, H, W, Cin, Cout, R, stride, pad,
                         (addend is not None, bool(accumulate), addend_mask is not None))):
            check(lib.mauv_conv2d_bwd_data_bn_h16(
                H16[w.dtype], _p(dy), _p(w), _p(dx), _p(addend), int(accumulate), G, B, H, W,
                Cin, Cout, R, R, stride, pad, _p(addend_mask), _p(b.get("y")), _p(b.get("out")),
                _p(mk),
                _p(b.get("scale")), _p(b.get("shift")), _p(b.get("mean")), _p(b.get("invstd")),
                int(b.get("relu", 0)), _p(b.get("p1")), _p(b.get("p2")), stream()),
                "conv2d_bwd_data_h16")
        return
    _f32(dy, w, dx, addend, b.get("y"), b.get("out"), b.get("scale"), b.get("shift"),
         b.get("mean"), b.get("invstd"), b.get("p1"), b.get("p2"))
    if b.get("mask") is not None:
        _dev(torch.uint8, b["mask"])
    if bn is not None:
        nb += 4 * G * B * H * W * Cin * (1 + (b.get("out") is not None))
    # a data gradient that also sums a BN's backward partials in its epilogue (engine
    # BWD_PARTIALS_F32) is its own kind in the bench's breakdown ("dgrad+bn"; inside the fp32
    # MFMA roofline, with the y bytes it reads counted)
    with _Prof("dgrad" if bn is None else "dgrad+bn", fl, nb, nl,
               info=(G, B, H, W, Cin, Cout, R, stride, pad,
                                           (addend is not None, bool(accumulate),
                                            addend_mask is not None))):
        check(lib.mauv_conv2d_bwd_data_f32(
            _p(dy), _p(w), _p(dx), _p(addend), _p(addend_mask), int(accumulate), G, B, H, W,
            Cin, Cout, R, R,
            stride, pad, _p(b.get("y")), _p(b.get("out")), _p(b.get("mask")), _p(b.get("scale")),
            _p(b.get("shift")), _p(b.get("mean")), _p(b.get("invstd")), int(b.get("relu", 0)),
            _p(b.get("p1")), _p(b.get("p2")), stream()), "conv2d_bwd_data")


def wgrad_splits(G, B, H, W, Cin, Cout, R, stride, pad):
    return lib.mauv_conv2d_wgrad_splits(G, B, H, W, Cin, Cout, R, R, stride, pad)


def conv2d_bwd_weight(x, dy, ws, splits, G, B, H, W, Cin, Cout, R, stride, pad,
                      x_strides=None, x_bn=None, alg_cin=None):
    """ws[splits][G][Cout][R*R*Cin] partial slabs (x' as in conv2d_fwd)."""
    xs = None if x_strides is None else _LL5(*x_strides)
    sc, sh, rl = x_bn if x_bn is not None else (None, None, 0)
    Ho, Wo = out_hw(H, R, stride, pad), out_hw(W, R, stride, pad)
    xg = 1 if (x_strides is not None and x_strides[0] == 0) else G
    fl = 2.0 * G * B * Ho * Wo * Cout * R * R * (alg_cin or Cin)
    nb = dy.element_size() * (xg * B * H * W * Cin + G * B * Ho * Wo * Cout) + 4.0 * ws.numel()
    if dy.dtype in H16:
        _h16(dy.dtype, dy)
        _f32(ws)
        assert x.is_cuda and x.dtype == dy.dtype and x.device.index == torch.cuda.current_device()
        with _Prof("wgrad_" + str(dy.dtype)[6:], fl, nb,
                   info=(G, B, H, W, Cin, Cout, R, stride, pad, x_bn is not None)):
            check(lib.mauv_conv2d_bwd_weight_h16(H16[dy.dtype], _p(x), xs, _p(sc), _p(sh), int(rl),
                                                 _p(dy), _p(ws), splits, G, B, H, W, Cin, Cout,
                                                 R, R, stride, pad, stream()),
                  "conv2d_bwd_weight_h16")
        return
    _f32(dy, ws)
    with _Prof("wgrad", fl, nb, info=(G, B, H, W, Cin, Cout, R, stride, pad, x_bn is not None)):
        check(lib.mauv_conv2d_bwd_weight_f32(_p(x), xs, _p(sc), _p(sh), int(rl), _p(dy), _p(ws),
                                             splits, G, B, H, W, Cin, Cout, R, R, stride, pad,
                                             stream()), "conv2d_bwd_weight")


# ----------------------------------------------------------------------- reparam / KL
def reparam_sample(mu, rho, out, G, seed, sample0, layer, Cout, Cin, RS, eps=None,
                   out_gstride=0, cin_pad=None):
    """out[g] (KRSC, group stride out_gstride or numel) = mu + softplus(rho) * eps_g.
    A bf16/f16 `out` gets 16-bit weights; cin_pad (>= Cin) channels in the KRSC layout (pad
    untouched) for the padded stems (8 channels 16-bit, 4 fp32)."""
    _f32(mu, rho, eps)
    if out.dtype in H16:
        check(lib.mauv_reparam_sample_h16(H16[out.dtype], _p(mu), _p(rho), _p(eps), seed, sample0,
                                          layer, G, Cout, Cin, RS, cin_pad or Cin, _p(out),
                                          out_gstride, stream()), "reparam_sample_h16")
        return
    if cin_pad not in (None, Cin):
        check(lib.mauv_reparam_sample_padded(_p(mu), _p(rho), _p(eps), seed, sample0, layer, G,
                                             Cout, Cin, RS, cin_pad, _p(out), out_gstride,
                                             stream()), "reparam_sample_padded")
        return
    check(lib.mauv_reparam_sample(_p(mu), _p(rho), _p(eps), seed, sample0, layer, G, Cout, Cin,
                                  RS, _p(out), out_gstride, stream()), "reparam_sample")


def reparam_sample_ex(mu, rho, out, G, seed, sample0, sample_base, layer, Cout, Cin, RS, eps=None,
                      out_gstride=0, cin_pad=None):
    """reparam_sample with the MC sample index sample0 + sample_base[0] + g read on the device
    (sample_base: int64 [1] device tensor) — what a replayed HIP graph of a forward uses."""
    _f32(mu, rho, eps)
    _dev(torch.int64, sample_base)
    code = -1 if out.dtype == torch.float32 else H16[out.dtype]
    check(lib.mauv_reparam_sample_ex(code, _p(mu), _p(rho), _p(eps), seed, sample0,
                                     _p(sample_base), layer, G, Cout, Cin, RS, cin_pad or Cin,
                                     _p(out), out_gstride, stream()), "reparam_sample_ex")


def reparam_bwd(dw, splits, mu, rho, dmu, drho, G, seed, sample0, layer, Cout, Cin, RS,
                eps=None, dw_gstride=0, dw_sstride=0, fixed_sample=-1, dw_cin=None):
    """fixed_sample >= 0: bayesian-torch semantics (rho-gradient uses that sample's eps for
    every MC group); -1: exact per-sample reparameterisation gradient.  dw_cin: channel count
    of the dw slabs' KRSC layout (the padded stems of the 16-bit path)."""
    _f32(mu, rho, dmu, drho, eps)   # dw may be a strided view (q|k|v slabs)
    check(lib.mauv_reparam_bwd(_p(dw), splits, dw_gstride, dw_sstride, _p(mu), _p(rho), _p(eps),
                               seed, sample0, layer, G, Cout, Cin, RS, dw_cin or Cin, _p(dmu),
                               _p(drho),
                               fixed_sample, stream()), "reparam_bwd")


def kl_fwd(table, n, workspace, out, scale=1.0):
    check(lib.mauv_kl_fwd(_p(table), n, _p(workspace), scale, _p(out), stream()), "kl_fwd")


def kl_bwd(table, n, coef=None, scale=1.0):
    check(lib.mauv_kl_bwd(_p(table), n, _p(coef), scale, stream()), "kl_bwd")


def philox_raw(seed, sample, layer, nq, device="cuda"):
    raw = torch.empty(nq * 4, dtype=torch.int32, device=device)
    nrm = torch.empty(nq * 4, dtype=torch.float32, device=device)
    check(lib.mauv_philox_raw(seed, sample, layer, nq, _p(raw), _p(nrm), stream()),
          "philox_raw")
    return raw, nrm


# ----------------------------------------------------------------------- batch norm
def bn_workspace_floats(G, M, C):
    return int(lib.mauv_bn_workspace_floats(G, M, C))


def bn_fwd_train(y, G, M, C, gamma, beta, run_mean, run_var, momentum, eps, ws, mean, invstd,
                 scale, shift, res, relu, out):
    _f32(y, gamma, beta, run_mean, run_var, ws, mean, invstd, scale, shift, res, out)
    check(lib.mauv_bn_fwd_train(_p(y), G, M, C, _p(gamma), _p(beta), _p(run_mean),
                                _p(run_var), momentum, eps, _p(ws), _p(mean), _p(invstd),
                                _p(scale), _p(shift), _p(res), int(relu), _p(out), stream()),
          "bn_fwd_train")


def bn_apply(y, scale, shift, res, relu, out, G, M, C, res_bn=None):
    """out = [relu](y*scale + shift (+ res')); res_bn = (res_scale, res_shift): the residual
    is a pending BN applied here (res' = res*res_scale + res_shift)."""
    rs, rh = res_bn if res_bn is not None else (None, None)
    if y.dtype in H16:
        _h16(y.dtype, y, res, out)
        check(lib.mauv_bn_apply_h16(H16[y.dtype], _p(y), _p(scale), _p(shift), _p(res), _p(rs),
                                    _p(rh), int(relu), _p(out), G, M, C, stream()), "bn_apply_h16")
        return
    _f32(y, res, out)
    check(lib.mauv_bn_apply(_p(y), _p(scale), _p(shift), _p(res), _p(rs), _p(rh), int(relu),
                            _p(out), G, M, C, stream()), "bn_apply")


def bn_eval_params(G, C, gamma, beta, run_mean, run_var, eps, scale, shift):
    check(lib.mauv_bn_eval_params(G, C, _p(gamma), _p(beta), _p(run_mean), _p(run_var), eps,
                                  _p(scale), _p(shift), stream()), "bn_eval_params")


def bn_stats_workspace_floats(G, nblk, C):
    return int(lib.mauv_bn_stats_workspace_floats(G, nblk, C))


def bn_stats_finalize(G, nblk, C, pmean, pm2, pcnt, gamma, beta, run_mean, run_var, momentum,
                      eps, ws, mean, invstd, scale, shift, ysh=None):
    """ysh: the centre the 16-bit forward stored y with (conv2d_fwd; its partials are those of
    the stored values): mean / shift describe the stored values, the running mean is updated
    with the true one (stored mean + ysh)."""
    _f32(ysh)
    check(lib.mauv_bn_stats_finalize(G, nblk, C, _p(pmean), _p(pm2), _p(pcnt), _p(gamma),
                                     _p(beta), _p(run_mean), _p(run_var), momentum, eps, _p(ws),
                                     _p(mean), _p(invstd), _p(scale), _p(shift), _p(ysh),
                                     stream()),
          "bn_stats_finalize")


def bn_bwd(y, out, dout, relu, mean, invstd, scale, G, M, C, ws, dy, dres=None, dgamma=None,
           dbeta=None, shift=None, pre=None):
    """out None + relu: mask from y*scale+shift.  pre = (p1, p2, nblk) partials from a dgrad
    epilogue (skips the partial pass)."""
    if y.dtype in H16:
        assert pre is None
        _h16(y.dtype, y, out, dout, dy, dres)
        _f32(mean, invstd, scale, shift, ws, dgamma, dbeta)
        check(lib.mauv_bn_bwd_h16(H16[y.dtype], _p(y), _p(out), _p(dout), int(relu), _p(mean),
                                  _p(invstd), _p(scale), _p(shift), G, M, C, _p(ws), _p(dy),
                                  _p(dres), _p(dgamma), _p(dbeta), stream()), "bn_bwd_h16")
        return
    _f32(y, out, dout, mean, invstd, scale, shift, ws, dy, dres, dgamma, dbeta)
    p1, p2, nb = pre if pre is not None else (None, None, 0)
    check(lib.mauv_bn_bwd(_p(y), _p(out), _p(dout), int(relu), _p(mean), _p(invstd), _p(scale),
                          _p(shift), G, M, C, _p(ws), _p(dy), _p(dres), _p(dgamma), _p(dbeta),
                          _p(p1), _p(p2), nb, stream()), "bn_bwd")


def bn_bwd_ex(y, out, mask, dout, relu, mean, invstd, scale, shift, G, M, C, ws, dy,
              dres=None, dgamma=None, dbeta=None, pre=None):
    """Every BN-backward form in one call: ReLU mask from `mask` bits (bn_apply_mask), else
    `out`, else y*scale+shift; pre = (p1, p2, nblk) partials a data-gradient epilogue wrote
    (conv2d_bwd_data(..., bn=...)) — the partial pass is skipped."""
    if y.dtype in H16:
        _h16(y.dtype, y, out, dout, dy, dres)
    else:
        _f32(y, out, dout, dy, dres)
    _f32(mean, invstd, scale, shift, ws, dgamma, dbeta)
    if mask is not None:
        _dev(torch.uint8, mask)
        if mask.numel() * 8 != G * M * C:
            raise ValueError("bn_bwd_ex: mask size does not match (G, M, C)")
    p1, p2, nb = pre if pre is not None else (None, None, 0)
    if pre is not None:
        _f32(p1, p2)
    check(lib.mauv_bn_bwd_ex(_dt_code(y), _p(y), _p(out), _p(mask), _p(dout), int(relu),
                             _p(mean), _p(invstd), _p(scale), _p(shift), G, M, C, _p(ws), _p(dy),
                             _p(dres), _p(dgamma), _p(dbeta), _p(p1), _p(p2), nb, stream()),
          "bn_bwd_ex")


def _dt_code(t):
    return -1 if t.dtype == torch.float32 else H16[t.dtype]


def bn_apply_mask(y, scale, shift, res, out, mask, G, M, C, res_bn=None):
    """bn_apply with relu, also writing the ReLU mask bits of out: mask uint8 [G*M*C/8]."""
    rs, rh = res_bn if res_bn is not None else (None, None)
    if mask.dtype != torch.uint8 or mask.numel() * 8 != G * M * C or out.numel() != G * M * C \
            or y.numel() != G * M * C or (res is not None and res.numel() != G * M * C):
        raise ValueError("bn_apply_mask: sizes do not match (G, M, C)")
    if y.dtype in H16:
        _h16(y.dtype, y, res, out)
    else:
        _f32(y, res, out)
    check(lib.mauv_bn_apply_mask(_dt_code(y), _p(y), _p(scale), _p(shift), _p(res), _p(rs),
                                 _p(rh), _p(out), _p(mask), G, M, C, stream()), "bn_apply_mask")


def bn_bwd_mask(y, mask, dout, mean, invstd, scale, G, M, C, ws, dy, dres=None, dgamma=None,
                dbeta=None):
    """BN + ReLU backward with the mask bits of bn_apply_mask in place of the output."""
    if mask.dtype != torch.uint8 or mask.numel() * 8 != G * M * C or dout.numel() != G * M * C:
        raise ValueError("bn_bwd_mask: sizes do not match (G, M, C)")
    if y.dtype in H16:
        _h16(y.dtype, y, dout, dy, dres)
    else:
        _f32(y, dout, dy, dres)
    _f32(mean, invstd, scale, ws, dgamma, dbeta)
    check(lib.mauv_bn_bwd_mask(_dt_code(y), _p(y), _p(mask), _p(dout), _p(mean), _p(invstd),
                               _p(scale), G, M, C, _p(ws), _p(dy), _p(dres), _p(dgamma),
                               _p(dbeta), stream()), "bn_bwd_mask")


# ----------------------------------------------------------------------- pooling
def maxpool_fwd(x, N, H, W, C, y, idx, bn=None):
    """3x3/2 pad-1 max-pool of N NHWC images; idx None skips the argmax bytes (no backward).
    bn = (scale, shift, G): x is the stem's conv output and relu(x*scale[g] + shift[g]) (its
    pending BatchNorm + ReLU, per MC group) is applied on load, never materialised."""
    Ho, Wo = out_hw(H, 3, 2, 1), out_hw(W, 3, 2, 1)
    if x.numel() != N * H * W * C or y.numel() != N * Ho * Wo * C or \
            (idx is not None and (idx.numel() != y.numel() or idx.dtype != torch.uint8)):
        raise ValueError("maxpool_fwd: tensor sizes do not match (N, H, W, C)")
    if bn is not None:
        scale, shift, G = bn
        if scale.numel() != G * C or shift.numel() != G * C or N % G:
            raise ValueError("maxpool_fwd: bn scale/shift must be [G][C] with G | N")
        if x.dtype in H16:
            _h16(x.dtype, x, y)
            check(lib.mauv_maxpool_bn_fwd_h16(H16[x.dtype], _p(x), _p(scale), _p(shift), G, N, H,
                                              W, C, _p(y), _p(idx), stream()), "maxpool_bn_fwd_h16")
            return
        _f32(x, y)
        check(lib.mauv_maxpool_bn_fwd(_p(x), _p(scale), _p(shift), G, N, H, W, C, _p(y), _p(idx),
                                      stream()), "maxpool_bn_fwd")
        return
    if x.dtype in H16:
        _h16(x.dtype, x, y)
        check(lib.mauv_maxpool_fwd_h16(H16[x.dtype], _p(x), N, H, W, C, _p(y), _p(idx), stream()),
              "maxpool_fwd_h16")
        return
    _f32(x, y)
    check(lib.mauv_maxpool_fwd(_p(x), N, H, W, C, _p(y), _p(idx), stream()), "maxpool_fwd")


def maxpool_bwd(dy, idx, N, H, W, C, dx):
    if dy.dtype in H16:
        _h16(dy.dtype, dy, dx)
        check(lib.mauv_maxpool_bwd_h16(H16[dy.dtype], _p(dy), _p(idx), N, H, W, C, _p(dx),
                                       stream()), "maxpool_bwd_h16")
        return
    _f32(dy, dx)
    check(lib.mauv_maxpool_bwd(_p(dy), _p(idx), N, H, W, C, _p(dx), stream()), "maxpool_bwd")


def avgpool_fwd(x, N, HW, C, y):
    """y fp32 [N][C] (pooled features feed the fp32 head) from fp32 or 16-bit x."""
    _f32(y)
    if x.dtype in H16:
        check(lib.mauv_avgpool_fwd_h16(H16[x.dtype], _p(x), N, HW, C, _p(y), stream()),
              "avgpool_fwd_h16")
        return
    check(lib.mauv_avgpool_fwd(_p(x), N, HW, C, _p(y), stream()), "avgpool_fwd")


def avgpool_bwd(dy, N, HW, C, dx):
    _f32(dy)
    if dx.dtype in H16:
        check(lib.mauv_avgpool_bwd_h16(H16[dx.dtype], _p(dy), N, HW, C, _p(dx), stream()),
              "avgpool_bwd_h16")
        return
    check(lib.mauv_avgpool_bwd(_p(dy), N, HW, C, _p(dx), stream()), "avgpool_bwd")


def pack_nchw(x, B, C, H, W, Cp, y):
    """fp32 NCHW images -> NHWC with Cp (zero-padded) channels: 16-bit (Cp 8) or fp32 (Cp 4)."""
    _f32(x)
    if y.dtype == torch.float32:
        check(lib.mauv_pack_nchw_f32(_p(x), B, C, H, W, Cp, _p(y), stream()), "pack_nchw_f32")
        return
    check(lib.mauv_pack_nchw_h16(H16[y.dtype], _p(x), B, C, H, W, Cp, _p(y), stream()),
          "pack_nchw_h16")


# ----------------------------------------------------------------------- stems (stem.hip)
def stem_kp(dtype, K):
    """Row width of the stem's im2col rows: K = Cin*R*S padded to the GEMM's K slice."""
    q = 32 if dtype == torch.float32 else 64
    return (K + q - 1) // q * q


def stem_im2col(x, B, C, H, W, R, stride, pad, Kp, cols):
    """cols[B*Ho*Wo][Kp] (fp32 / bf16 / f16) from fp32 NCHW images, k = c*R*R + r*R + s."""
    _f32(x)
    assert cols.is_cuda and cols.is_contiguous()
    code = -1 if cols.dtype == torch.float32 else H16[cols.dtype]
    Ho, Wo = out_hw(H, R, stride, pad), out_hw(W, R, stride, pad)
    assert cols.numel() == B * Ho * Wo * Kp
    check(lib.mauv_stem_im2col(code, _p(x), B, C, H, W, R, R, stride, pad, Kp, _p(cols),
                               stream()), "stem_im2col")


def stem_fwd(cols, w, y, G, M, Kp, Cout, stats, alg_k, ysh=None):
    """y[G][M][Cout] = cols[M][Kp] . w[g][Cout][Kp]^T for every g as one GEMM (weights stacked
    along N); stats = (mean, m2, cnt) partials as conv2d_fwd's.  alg_k: the stem's real
    Cin*R*S (profiling counts algorithmic work, not the zero padding).  ysh: centred storage
    (16-bit only, conv2d_fwd's)."""
    sm, s2, sn = stats
    fl = 2.0 * G * M * Cout * alg_k
    esz = w.element_size()
    nb = esz * (M * Kp + G * Cout * Kp + G * M * Cout)
    if w.dtype in H16:
        _h16(w.dtype, cols, w, y)
        _f32(ysh)
        with _Prof("fwd_" + str(w.dtype)[6:], fl, nb, info=("stem", G, M, Kp, Cout)):
            check(lib.mauv_stem_fwd_h16(H16[w.dtype], _p(cols), _p(w), _p(y), G, M, Kp, Cout,
                                        _p(sm), _p(s2), _p(sn), _p(ysh), stream()),
                  "stem_fwd_h16")
        return
    if ysh is not None:
        raise ValueError("stem_fwd: ysh (centred storage) is for the 16-bit stems")
    _f32(cols, w, y)
    with _Prof("fwd", fl, nb, info=("stem", G, M, Kp, Cout)):
        check(lib.mauv_stem_fwd_f32(_p(cols), _p(w), _p(y), G, M, Kp, Cout, _p(sm), _p(s2),
                                    _p(sn), stream()), "stem_fwd_f32")


# ----------------------------------------------------------------------- head
def attn_t(qkv, rows, hid, t):
    _dev(torch.float32, qkv, t)
    check(lib.mauv_attn_t(_p(qkv), rows, hid, _p(t), stream()), "attn_t")


def attn_t_bwd(dt, t, rows, hid, dqkv):
    _dev(torch.float32, dt, t, dqkv)
    check(lib.mauv_attn_t_bwd(_p(dt), _p(t), rows, hid, _p(dqkv), stream()), "attn_t_bwd")


def attn_out(qkv, s, rows, hid, comb, ld, off):
    _dev(torch.float32, qkv, s, comb)
    check(lib.mauv_attn_out(_p(qkv), _p(s), rows, hid, _p(comb), ld, off, stream()),
          "attn_out")


def attn_out_bwd(dcomb, ld, off, qkv, s, rows, hid, dqkv, ds):
    _dev(torch.float32, dcomb, qkv, s, dqkv, ds)
    check(lib.mauv_attn_out_bwd(_p(dcomb), ld, off, _p(qkv), _p(s), rows, hid, _p(dqkv),
                                _p(ds), stream()), "attn_out_bwd")


def colsum(dy, G, rows, N, out, accumulate=False):
    _dev(torch.float32, dy, out)
    check(lib.mauv_colsum(_p(dy), G, rows, N, _p(out), int(accumulate), stream()), "colsum")


def mc_mean_ce(logits, labels, G, B, C, mean, loss, pred=None):
    _dev(torch.float32, logits, mean, loss)
    _dev(torch.int64, labels, pred)
    check(lib.mauv_mc_mean_ce(_p(logits), _p(labels), G, B, C, _p(mean), _p(loss), _p(pred),
                              stream()), "mc_mean_ce")


def mc_mean_bwd(dmean, gloss, mean, labels, G, B, C, dlogits):
    _dev(torch.float32, dmean, gloss, mean, dlogits)
    _dev(torch.int64, labels)
    check(lib.mauv_mc_mean_bwd(_p(dmean), _p(gloss), _p(mean), _p(labels), G, B, C,
                               _p(dlogits), stream()), "mc_mean_bwd")


def mc_stats(logits, G, B, C, eps_h, sums, accumulate=False):
    _dev(torch.float32, logits)
    _dev(torch.float64, sums)
    check(lib.mauv_mc_stats(_p(logits), G, B, C, eps_h, _p(sums), int(accumulate), stream()),
          "mc_stats")


def mc_finalize(sums, N, B, C, eps_pred, mean_prob=None, var_unc=None, alea=None,
                pred_entropy=None, pred=None):
    _dev(torch.float64, sums)
    _dev(torch.float32, mean_prob, var_unc, alea, pred_entropy)
    _dev(torch.int64, pred)
    check(lib.mauv_mc_finalize(_p(sums), N, B, C, eps_pred, _p(mean_prob), _p(var_unc),
                               _p(alea), _p(pred_entropy), _p(pred), stream()), "mc_finalize")


def nonfinite_count(t, out):
    _dev(torch.float32, t)
    _dev(torch.int32, out)
    check(lib.mauv_nonfinite_count(_p(t), t.numel(), _p(out), stream()), "nonfinite_count")
