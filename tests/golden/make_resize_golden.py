"""Golden vectors for the device Resize (data/datasets.py:240-246: transforms.Resize on a PIL
tile = PIL Image.resize(size, BILINEAR)).  Run here, where Pillow is importable:

    python tests/golden/make_resize_golden.py

writes tests/golden/resize_golden.npz: seeded uint8 tiles and Pillow's resized outputs
(downscales with antialiasing, upscales, one-axis changes, 1- and 3-channel).  The fixture
records the Pillow version it was made with; the reference pins pillow 11.0.0."""
import os

import numpy as np
from PIL import Image, __version__ as PIL_VERSION

CASES = [  # H, W, C, Ho, Wo
    (37, 53, 3, 24, 40),      # downscale, two different factors
    (20, 30, 1, 64, 48),      # upscale (grayscale SSS-like tile)
    (100, 77, 3, 40, 40),     # 2.5x / 1.9x downscale
    (33, 64, 3, 33, 16),      # width only
    (16, 16, 1, 47, 16),      # height only, upscale
]


def pil_resize(a, Ho, Wo):
    C = a.shape[2]
    im = Image.fromarray(a[:, :, 0] if C == 1 else a, "L" if C == 1 else "RGB")
    r = np.asarray(im.resize((Wo, Ho), Image.BILINEAR))
    return r[:, :, None] if C == 1 else r


def main():
    rng = np.random.default_rng(2024)
    out = {"pillow_version": np.array(PIL_VERSION)}
    for i, (H, W, C, Ho, Wo) in enumerate(CASES):
        a = rng.integers(0, 256, (H, W, C), dtype=np.uint8)
        out[f"in{i}"] = a
        out[f"out{i}"] = pil_resize(a, Ho, Wo)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "resize_golden.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} (Pillow {PIL_VERSION})")


if __name__ == "__main__":
    main()
