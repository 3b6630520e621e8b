"""Accuracy of the fp32 conv arithmetics vs float64: max |err| / max |ref| of fwd y, dgrad dx
and wgrad dW per mode, on a few ResNet-50 shapes.

    python tools/f32_math_diag.py [modes, default exact,split,split1,split3]
"""
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd")]
import torch  # noqa: E402

from tests.test_f32_math_gpu import _ref_all, _run_all  # noqa: E402
from mauv import ops  # noqa: E402

CASES = [(2, 2, 8, 64, 64, 3, 1, 1), (1, 4, 14, 256, 256, 3, 1, 1), (2, 2, 4, 512, 2048, 1, 1, 0),
         (1, 8, 16, 128, 512, 1, 1, 0)]


def main():
    modes = (sys.argv[1] if len(sys.argv) > 1 else "exact,split,split1,split3").split(",")
    for case in CASES:
        G, B, H, Cin, Cout, R, st, pad = case
        torch.manual_seed(0)
        x = torch.randn(G, B, H, H, Cin)
        w = torch.randn(G, Cout, R, R, Cin) / math.sqrt(Cin * R * R)
        Ho = (H + 2 * pad - R) // st + 1
        dy = torch.randn(G, B, Ho, Ho, Cout)
        refs = _ref_all(x, w, dy, st, pad)
        row = []
        for m in modes:
            ops.set_f32_math(m)
            outs = _run_all(x, w, dy, G, B, H, Cin, Cout, R, st, pad)
            row.append(m + " " + " ".join(
                f"{(o.double() - r).abs().max().item() / r.abs().max().item():.2e}"
                for o, r in zip(outs, refs)))
        print(case, " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
