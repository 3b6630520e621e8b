"""Probe: the 16-bit implicit-GEMM conv (mauv conv_pipe16, statistics epilogue on) against the
library GEMM (torch.bmm -> hipBLASLt) on the same M x N x K, per ResNet-50 1x1 / 3x3 shape.
Measurement only (not on the product path).

    python tools/gemm_probe.py [--G 10] [--B 256] [--dtype f16]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd")]
import torch  # noqa: E402
from mauv import ops  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--G", type=int, default=10)
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--dtype", default="f16", choices=["bf16", "f16"])
    a = ap.parse_args()
    dt = {"bf16": torch.bfloat16, "f16": torch.float16}[a.dtype]
    G, B = a.G, a.B
    shapes = []
    for S in (224, 256):
        h = S // 4
        for (cin, cout, r, hh) in ((64, 64, 1, h), (256, 64, 1, h), (64, 256, 1, h), (64, 64, 3, h),
                                   (256, 128, 1, h), (512, 128, 1, h // 2), (128, 128, 3, h // 2),
                                   (128, 512, 1, h // 2), (512, 256, 1, h // 2),
                                   (1024, 256, 1, h // 4), (256, 256, 3, h // 4),
                                   (256, 1024, 1, h // 4), (1024, 512, 1, h // 4),
                                   (2048, 512, 1, h // 8), (512, 512, 3, h // 8),
                                   (512, 2048, 1, h // 8)):
            shapes.append((S, cin, cout, r, hh))
    print(f"{'S':>4s} {'Cin':>5s} {'Cout':>5s} {'R':>2s} {'H':>3s} {'conv ms':>8s} {'TF/s':>6s} "
          f"{'bmm ms':>8s} {'TF/s':>6s}")
    tc = tb = 0.0
    for S, cin, cout, r, hh in shapes:
        pd = r // 2
        x = torch.randn(G, B, hh, hh, cin, device="cuda").to(dt)
        w = (torch.randn(G, cout, r, r, cin, device="cuda") * 0.05).to(dt)
        y = torch.empty(G, B, hh, hh, cout, device="cuda", dtype=dt)
        nblk = ops.fwd_stat_blocks(G, B, hh, hh, cin, cout, r, 1, pd)
        st = (torch.empty(G, nblk, cout, device="cuda"), torch.empty(G, nblk, cout, device="cuda"),
              torch.empty(G, nblk, device="cuda"))
        fl = 2.0 * G * B * hh * hh * cout * r * r * cin
        t1 = timeit(lambda: ops.conv2d_fwd(x, w, y, G, B, hh, hh, cin, cout, r, 1, pd, stats=st))
        M, K = B * hh * hh, r * r * cin
        A = torch.randn(G, M, K, device="cuda").to(dt)
        Wt = (torch.randn(G, K, cout, device="cuda") * 0.05).to(dt)
        C = torch.empty(G, M, cout, device="cuda", dtype=dt)
        t2 = timeit(lambda: torch.bmm(A, Wt, out=C))
        tc += t1
        tb += t2
        print(f"{S:4d} {cin:5d} {cout:5d} {r:2d} {hh:3d} {t1:8.3f} {fl / t1 / 1e9:6.0f} {t2:8.3f} "
              f"{fl / t2 / 1e9:6.0f}", flush=True)
        del x, w, y, A, Wt, C, st
        torch.cuda.empty_cache()
    print(f"TOTAL conv {tc:.2f} ms, bmm {tb:.2f} ms")


if __name__ == "__main__":
    main()
