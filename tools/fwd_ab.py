"""A/B/C of the 16-bit forward kernels over every conv of the three trunks (the bench's training
slice G=5, B=64 by default; --G 50 --B 256 ~ an f16 inference chunk): the library's routing
("route": conv_big16 / conv_expand16 / conv_haloc16 / conv_halo16 where the measured rules send a
shape), conv_big16's 256-row LDS-DMA tiles on every covered shape ("big16") and the implicit GEMM
alone ("pipe16"), interleaved rounds in one process, with the pending BN on load where the engine
has it (conv2, conv3) and the statistics epilogue; and, for the 1x1 / stride-1 shapes, the vendor
GEMM on the same operands ("bmm": torch.bmm [G, M, K] x [G, K, N] through --blas, without the
BN transform or the statistics the conv kernels also do).

    python tools/fwd_ab.py [--dtype bf16|f16] [--G 5] [--B 64] [--min-k 512 (the minimum)] [--rounds 3]
                           [--blas hipblaslt|rocblas] [--only1x1]
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
    ap.add_argument("--blas", default="hipblaslt", choices=["hipblaslt", "rocblas"])
    ap.add_argument("--only1x1", action="store_true")
    a = ap.parse_args()
    torch.backends.cuda.preferred_blas_library("cublaslt" if a.blas == "hipblaslt" else "cublas")
    dt = {"bf16": torch.bfloat16, "f16": torch.float16}[a.dtype]
    G, B, dev = a.G, a.B, "cuda"
    torch.manual_seed(0)
    shapes = {}
    for trunk, cin, S in (("opt", 3, 224), ("bathy", 3, 256), ("sss", 1, 256)):
        for name, Cin, Cout, R, st, pd, H in trunk_convs(cin, S):
            if name == "stem" or Cin * R * R < a.min_k or (a.only1x1 and R != 1):
                continue
            key = (Cin, Cout, R, st, pd, H, name.endswith(("c2", "c3")))
            shapes.setdefault(key, []).append(f"{trunk}:{name}")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ARMS = ("route", "pipe16", "big16", "bmm")
    res = {k: {arm: [] for arm in ARMS} for k in shapes}
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
            order = ARMS[rnd % 4:] + ARMS[:rnd % 4]
            for arm in order:
                if arm == "bmm" and (R != 1 or st != 1):
                    res[key][arm].append(float("nan"))
                    continue
                prev = ops.route()
                if arm == "pipe16":
                    ops.set_route(big16=0, expand16=0, haloc16=0, halo3=0)
                elif arm == "big16":
                    ops.set_route(big16=2, big16_min_k=a.min_k)
                try:
                    if arm == "bmm":
                        A2 = x.view(G, B * H * H, Cin)
                        W2 = w.view(G, Cout, Cin).transpose(1, 2)
                        fn = lambda: torch.bmm(A2, W2)
                    else:
                        fn = lambda: ops.conv2d_fwd(x, w, y, G, B, H, H, Cin, Cout, R, st, pd,
                                                    x_bn=x_bn, stats=stats)
                    fn()
                    torch.cuda.synchronize()
                    e0.record()
                    for _ in range(a.reps):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    res[key][arm].append(e0.elapsed_time(e1) / a.reps)
                finally:
                    ops.set_route(**prev)
            del x, w, y
    tot = {arm: 0.0 for arm in ARMS}
    print(f"{'Cin,Cout,R,s,H,xbn':28s} {'n':>3s} " + " ".join(f"{x + ' ms':>11s}" for x in ARMS) +
          " " + " ".join(f"{'TF/s ' + x:>12s}" for x in ARMS) + "  layers")
    for key, v in sorted(shapes.items(), key=lambda kv: -min(res[kv[0]]["route"])):
        Cin, Cout, R, st, pd, H, xb = key
        Ho = ops.out_hw(H, R, st, pd)
        fl = 2.0 * G * B * Ho * Ho * Cout * R * R * Cin
        t = {arm: min(res[key][arm]) for arm in ARMS}
        for arm in ARMS:
            tot[arm] += (t[arm] if t[arm] == t[arm] else t["route"]) * len(v)
        print(f"{str((Cin, Cout, R, st, H, int(xb))):28s} {len(v):3d} " +
              " ".join(f"{t[x]:11.3f}" for x in ARMS) + " " +
              " ".join(f"{fl / t[x] / 1e9:12.0f}" for x in ARMS) + f"  {' '.join(v[:4])}")
    print("TOTAL (x occurrences; bmm: the route's time where it does not apply): " +
          ", ".join(f"{x} {tot[x]:.2f} ms" for x in ARMS))

if __name__ == "__main__":
    main()
