"""A/B of the 16-bit forward kernels over every conv of the three trunks (the bench's training
slice G=5, B=64 by default; --G 50 --B 256 ~ an f16 inference chunk): conv_big16 (256-row
LDS-DMA tiles) against the implicit GEMM (conv_pipe16), interleaved rounds in one process, with
the pending BN on load where the engine has it (conv2, conv3) and the statistics epilogue.

    python tools/fwd_ab.py [--dtype bf16|f16] [--G 5] [--B 64] [--min-k 512] [--rounds 3]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd"), os.path.join(REPO, "tools")]
import torch  # noqa: E402
from mauv import ops  # noqa: E402
from conv_bench import trunk_convs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16"])
    ap.add_argument("--G", type=int, default=5)
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--min-k", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dt = {"bf16": torch.bfloat16, "f16": torch.float16}[a.dtype]
    G, B, dev = a.G, a.B, "cuda"
    torch.manual_seed(0)
    shapes = {}
    for trunk, cin, S in (("opt", 3, 224), ("bathy", 3, 256), ("sss", 1, 256)):
        for name, Cin, Cout, R, st, pd, H in trunk_convs(cin, S):
            if name == "stem" or Cin * R * R < a.min_k:
                continue
            key = (Cin, Cout, R, st, pd, H, name.endswith(("c2", "c3")))
            shapes.setdefault(key, []).append(f"{trunk}:{name}")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {k: {True: [], False: []} for k in shapes}
    for rnd in range(a.rounds):
        for key in shapes:
            Cin, Cout, R, st, pd, H, xb = key
            Ho = ops.out_hw(H, R, st, pd)
            x = torch.randn(G, B, H, H, Cin, device=dev).to(dt)
            w = (torch.randn(G, Cout, R, R, Cin, device=dev) * 0.05).to(dt)
            y = torch.empty(G, B, Ho, Ho, Cout, device=dev, dtype=dt)
            nblk = ops.fwd_stat_blocks(G, B, H, H, Cin, Cout, R, st, pd)
            stats = tuple(torch.empty(*s, device=dev) for s in ((G, nblk, Cout), (G, nblk, Cout),
                                                               (G, nblk)))
            x_bn = (torch.rand(G, Cin, device=dev) + 0.5, torch.randn(G, Cin, device=dev) * 0.1,
                    1) if xb else None
            for big in ((True, False) if rnd % 2 == 0 else (False, True)):
                prev = ops.set_big16(2 if big else 0, a.min_k)
                try:
                    fn = lambda: ops.conv2d_fwd(x, w, y, G, B, H, H, Cin, Cout, R, st, pd,
                                                x_bn=x_bn, stats=stats)
                    fn()
                    e0.record()
                    for _ in range(a.reps):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    res[key][big].append(e0.elapsed_time(e1) / a.reps)
                finally:
                    ops.set_big16(prev)
            del x, w, y
    tot = {True: 0.0, False: 0.0}
    print(f"{'Cin,Cout,R,s,H,xbn':28s} {'n':>3s} {'pipe16 ms':>10s} {'big16 ms':>10s} {'ratio':>6s} "
          f"{'TF/s pipe':>9s} {'TF/s big':>9s}  layers")
    for key, v in sorted(shapes.items(), key=lambda kv: -min(res[kv[0]][False])):
        Cin, Cout, R, st, pd, H, xb = key
        Ho = ops.out_hw(H, R, st, pd)
        fl = 2.0 * G * B * Ho * Ho * Cout * R * R * Cin
        tb, tp = min(res[key][True]), min(res[key][False])
        tot[True] += tb * len(v)
        tot[False] += tp * len(v)
        print(f"{str((Cin, Cout, R, st, H, int(xb))):28s} {len(v):3d} {tp:10.3f} {tb:10.3f} "
              f"{tb / tp:6.3f} {fl / tp / 1e9:9.0f} {fl / tb / 1e9:9.0f}  {' '.join(v[:4])}")
    print(f"TOTAL (x occurrences): pipe16 {tot[False]:.2f} ms, big16 {tot[True]:.2f} ms, "
          f"ratio {tot[True] / tot[False]:.3f}")


if __name__ == "__main__":
    main()
