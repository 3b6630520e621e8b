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
