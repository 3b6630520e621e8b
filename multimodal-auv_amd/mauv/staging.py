"""Input staging on the device through libmauv_hip (staging.hip).

* ``to_tensor_normalize(tiles_u8, mean, std)``: the per-tile transforms of
  data/datasets.py:239-250 — ``ToTensor`` (x / 255, HWC -> CHW) and, for the optical tiles,
  ``Normalize(mean, std)`` — on a batch of decoded uint8 tiles [B, H, W, C] (PIL's layout),
  bit-exact with torchvision's fp32 ops.  Copying the uint8 tiles to the GPU moves a quarter
  of the bytes the reference's fp32 tensors do (train/multimodal.py:87-94).
* ``simulate_underwater_degradation(clean_image, uniform_distance_map, turbidity_factor,
  depth_value)``: the underwater image formation model of
  Examples/"Example training with image noise.py":55-93, same signature and maths, one
  fused element-wise kernel; ``to_tensor_normalize(..., degrade=(turbidity, depth, map))``
  applies it in the same pass as the normalisation.

Tensors must be on a ROCm device (no host path: the reference's own torch code is the
CPU path).
"""
import numpy as np
import torch

from . import ops
from ._lib import lib, check

# data/datasets.py:244-249 (transform_1 of the optical tiles)
OPTICAL_MEAN = (62.19902423 / 255.0, 62.31835042 / 255.0, 61.53444229 / 255.0)
OPTICAL_STD = (41.46890313 / 255.0, 43.39430715 / 255.0, 41.72083641 / 255.0)
# datasets.py:240/244: every tile is resized to 256 x 256
TILE_SIZE = (256, 256)
# Example training with image noise.py:70-79: attenuation per channel and backscatter light
UIFM_BETA = (0.8, 0.5, 0.3)
UIFM_BINF = (0.1, 0.3, 0.5)


def _f32_dev(vals, dev):
    return torch.tensor(np.asarray(vals, dtype=np.float32), device=dev)


def _uifm_params(C, turbidity_factor, dev):
    if C != len(UIFM_BETA):
        raise ValueError(f"UIFM degradation is defined for {len(UIFM_BETA)}-channel images "
                         f"(got {C}), as in the reference (beta.view(1, C, 1, 1))")
    # the reference: torch.tensor(beta, dtype=float32) * turbidity -> fp32 products
    bt = np.asarray(UIFM_BETA, dtype=np.float32) * np.float32(turbidity_factor)
    return _f32_dev(bt, dev), _f32_dev(UIFM_BINF, dev)


def _dist(dist, B, H, W, dev):
    if dist is None:
        return None
    if dist.numel() != B * H * W:
        raise ValueError("distance map must be [B, 1, H, W]")
    d = dist.to(dev, torch.float32).contiguous()
    if torch.all(d == 1).item():
        return None          # the reference's uniform map: no per-pixel read
    return d


def to_tensor_normalize(tiles, mean=None, std=None, degrade=None, out=None):
    """uint8 [B, H, W, C] tiles -> fp32 [B, C, H, W] on the GPU: x / 255, then
    (x - mean) / std when given; degrade = (turbidity_factor, depth_value[, distance_map])
    applies the UIFM degradation to the result in the same pass."""
    if tiles.dtype != torch.uint8 or tiles.dim() != 4:
        raise ValueError("tiles must be uint8 [B, H, W, C]")
    if not tiles.is_cuda:
        raise ValueError("tiles must be on a ROCm device (copy the uint8 batch, 4x fewer bytes)")
    tiles = tiles.contiguous()
    B, H, W, C = tiles.shape
    dev = tiles.device
    out = torch.empty(B, C, H, W, device=dev) if out is None else out
    ops._dev(torch.float32, out)
    m = s = bt = binf = dist = None
    if mean is not None:
        m, s = _f32_dev(mean, dev), _f32_dev(std, dev)
    depth = 1.0
    if degrade is not None:
        turb, depth = degrade[0], float(degrade[1])
        bt, binf = _uifm_params(C, turb, dev)
        dist = _dist(degrade[2] if len(degrade) > 2 else None, B, H, W, dev)
    check(lib.mauv_stage_u8(tiles.data_ptr(), B, H, W, C, ops._p(m), ops._p(s), ops._p(bt),
                            ops._p(binf), ops._p(dist), depth, out.data_ptr(), ops.stream()),
          "stage_u8")
    return out


def resize(tiles, size=(256, 256), mean=None, std=None, degrade=None):
    """data/datasets.py:240-246 on the device: ``transforms.Resize(size)`` of decoded uint8
    tiles [B, H, W, C] (PIL's Image.resize(BILINEAR), bit-exact with Pillow's 8-bit
    resampler), returned as uint8 [B, Ho, Wo, C] — or, with ``mean``/``std`` and/or
    ``degrade`` given (or ``to_tensor=True`` via :func:`resize_to_tensor`), ToTensor /
    Normalize / UIFM applied in the same pass into fp32 [B, C, Ho, Wo]."""
    return _resize(tiles, size, mean, std, degrade, staged=mean is not None or degrade is not None)


def resize_to_tensor(tiles, size=(256, 256), mean=None, std=None, degrade=None):
    """``Compose([Resize(size), ToTensor(), Normalize(mean, std)])`` (datasets.py:243-250) on the
    device: uint8 [B, H, W, C] -> fp32 [B, C, Ho, Wo] in one resize pass + the staging maths."""
    return _resize(tiles, size, mean, std, degrade, staged=True)


def _resize(tiles, size, mean, std, degrade, staged):
    if tiles.dtype != torch.uint8 or tiles.dim() != 4:
        raise ValueError("tiles must be uint8 [B, H, W, C]")
    if not tiles.is_cuda:
        raise ValueError("tiles must be on a ROCm device")
    tiles = tiles.contiguous()
    B, H, W, C = tiles.shape
    Ho, Wo = (size, size) if isinstance(size, int) else size
    dev = tiles.device
    nws = int(lib.mauv_resize_workspace_bytes(B, H, W, C, Ho, Wo))
    if nws < 0:
        raise ValueError(f"resize: unsupported shape {tuple(tiles.shape)} -> {(Ho, Wo)}")
    ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=dev)
    m = s = bt = binf = dist = None
    depth = 1.0
    if staged:
        out = torch.empty(B, C, Ho, Wo, device=dev)
        if mean is not None:
            m, s = _f32_dev(mean, dev), _f32_dev(std, dev)
        if degrade is not None:
            turb, depth = degrade[0], float(degrade[1])
            bt, binf = _uifm_params(C, turb, dev)
            dist = _dist(degrade[2] if len(degrade) > 2 else None, B, Ho, Wo, dev)
        o8, of = None, out
    else:
        out = torch.empty(B, Ho, Wo, C, dtype=torch.uint8, device=dev)
        o8, of = out, None
    check(lib.mauv_resize_u8(tiles.data_ptr(), B, H, W, C, Ho, Wo, ws.data_ptr(), ops._p(o8),
                             ops._p(m), ops._p(s), ops._p(bt), ops._p(binf), ops._p(dist), depth,
                             ops._p(of), ops.stream()), "resize_u8")
    return out


def simulate_underwater_degradation(clean_image, uniform_distance_map, turbidity_factor,
                                    depth_value):
    """Examples/"Example training with image noise.py":55-93 on the GPU (fp32 NCHW)."""
    if not clean_image.is_cuda:
        raise ValueError("clean_image must be on a ROCm device")
    x = clean_image.contiguous().float()
    B, C, H, W = x.shape
    bt, binf = _uifm_params(C, turbidity_factor, x.device)
    dist = _dist(uniform_distance_map, B, H, W, x.device)
    out = torch.empty_like(x)
    check(lib.mauv_uifm(x.data_ptr(), B, C, H, W, bt.data_ptr(), binf.data_ptr(), ops._p(dist),
                        float(depth_value), out.data_ptr(), ops.stream()), "uifm")
    return out.to(clean_image.dtype)


def stage_tile_batch(t, optical):
    """A batch tensor as the drop-in loops receive it: fp32 tiles (the reference's datasets
    already applied their transforms on the host) pass through; decoded uint8 HWC tiles
    [B, H, W, C] (C = 1 or 3) on the device get datasets.py:239-250's transforms here —
    Resize((256, 256)), ToTensor and, for the optical tile, Normalize — in one pass."""
    if t.dtype != torch.uint8 or t.dim() != 4 or t.shape[-1] not in (1, 3) or not t.is_cuda:
        return t
    if optical:
        return resize_to_tensor(t, TILE_SIZE, OPTICAL_MEAN, OPTICAL_STD)
    return resize_to_tensor(t, TILE_SIZE)
