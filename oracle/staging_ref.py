"""Oracle: the reference's input transforms and UIFM degradation (TEST INFRASTRUCTURE ONLY).

* ``to_tensor_normalize``  data/datasets.py:239-250: torchvision ToTensor on a PIL image
  (``img.float().div(255)`` after HWC -> CHW) and Normalize (``tensor.sub_(mean).div_(std)``
  with fp32 mean/std) — restated with the same torch fp32 ops on a uint8 [B, H, W, C] batch.
* ``simulate_underwater_degradation``  Examples/"Example training with image noise.py":55-93,
  restated op for op (beta * turbidity, map * depth, exp(-beta * d), J * t + B_inf * (1 - t),
  clamp to [0, 1]).
"""
import torch


def to_tensor_normalize(tiles_u8, mean=None, std=None):
    x = tiles_u8.permute(0, 3, 1, 2).contiguous().to(torch.float32).div(255)
    if mean is not None:
        m = torch.as_tensor(mean, dtype=torch.float32).view(1, -1, 1, 1)
        s = torch.as_tensor(std, dtype=torch.float32).view(1, -1, 1, 1)
        x = x.sub(m).div(s)
    return x


def simulate_underwater_degradation(clean_image, uniform_distance_map, turbidity_factor,
                                    depth_value):
    B, C, H, W = clean_image.shape
    beta = torch.tensor([0.8, 0.5, 0.3], dtype=clean_image.dtype).view(1, C, 1, 1) \
        * turbidity_factor
    B_inf = torch.tensor([0.1, 0.3, 0.5], dtype=clean_image.dtype).view(1, C, 1, 1)
    d = uniform_distance_map * depth_value
    t = torch.exp(-beta * d.expand(B, C, H, W))
    return torch.clamp(clean_image * t + B_inf * (1.0 - t), 0.0, 1.0)


# ---------------------------------------------------------------------------- Resize
# data/datasets.py:240-246: transforms.Resize((256, 256)) on the PIL tile, i.e. PIL's
# Image.resize(size, BILINEAR) (torchvision passes PIL images to PIL; PIL always antialiases).
# Restated from Pillow's 8-bit separable resampler (libImaging/Resample.c, the reference pins
# pillow 11.0.0): double-precision normalised triangle-filter coefficients whose support grows
# with the downscale factor, converted to 22-bit fixed point; a horizontal pass into an 8-bit
# intermediate image (round half up via the 2^21 bias, floor shift, clamp to 0..255), then the
# vertical pass the same way.  Pinned against PIL itself (tests/golden/make_resize_golden.py).
PRECISION_BITS = 32 - 8 - 2


def _bilinear(x):
    x = abs(x)
    return 1.0 - x if x < 1.0 else 0.0


def resize_coeffs(in_size, out_size):
    """(bounds [out][2] = (xmin, n), fixed-point coefficients [out][ksize]) as Resample.c's
    precompute_coeffs + normalize_coeffs_8bpc for box (0, in_size)."""
    import math
    import numpy as np
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    ss = 1.0 / filterscale
    bounds = np.zeros((out_size, 2), np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        w = [_bilinear((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for v in w:
            ww += v
        for x in range(xmax):
            k = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = int(-0.5 + k * (1 << PRECISION_BITS)) if k < 0 else \
                int(0.5 + k * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _pass(img, bounds, kk, axis):
    """One 8-bit pass along ``axis`` (1 = width, 0 = height) of an [H, W, C] uint8 image."""
    import numpy as np
    src = np.moveaxis(img.astype(np.int64), axis, 0)       # [in, other, C]
    out = np.zeros((bounds.shape[0],) + src.shape[1:], np.int64)
    for o, (xmin, n) in enumerate(bounds):
        acc = np.full(src.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
        for x in range(n):
            acc += src[xmin + x] * kk[o, x]
        out[o] = np.clip(acc >> PRECISION_BITS, 0, 255)
    return np.moveaxis(out, 0, axis).astype(np.uint8)


def pil_resize_bilinear(img_hwc, out_h, out_w):
    """uint8 [H, W, C] -> uint8 [out_h, out_w, C] as PIL's Image.resize((out_w, out_h),
    BILINEAR): horizontal pass first (when the width changes), then vertical."""
    H, W = img_hwc.shape[:2]
    x = img_hwc
    if out_w != W:
        x = _pass(x, *resize_coeffs(W, out_w), axis=1)
    if out_h != H:
        x = _pass(x, *resize_coeffs(H, out_h), axis=0)
    return x
