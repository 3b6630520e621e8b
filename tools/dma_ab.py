"""Per-shape A/B of the LDS-DMA 16-bit conv kernels (conv_dma16.hip) against the pipelined
register-staged ones (conv_pipe16.hip), interleaved in one process so that clock and box
drift cancel: every unique conv shape of the three trunks at the bench's training slice
(G=5 MC groups, B=64, 224 optical / 256 sonar), forward without and with a pending BN on x,
and the data gradient (DMA over the RSCK-transposed weights, the transpose timed apart).

    python tools/dma_ab.py [--dtype bf16|f16] [--G 5] [--B 64] [--rounds 3]
"""
import argparse
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd"), os.path.join(REPO, "tools")]
import torch  # noqa: E402
from mauv import ops  # noqa: E402
from conv_bench import trunk_convs  # noqa: E402


def timeit(fn, reps):
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
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16"])
    ap.add_argument("--G", type=int, default=5)
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--passes", default="fwd,fwdbn,dgrad")
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    G, B, dev = a.G, a.B, "cuda"
    shapes = defaultdict(int)   # unique shape -> multiplicity over the three trunks
    for cin, S in ((3, 224), (3, 256), (1, 256)):
        for name, Cin, Cout, R, st, pd, H in trunk_convs(cin, S):
            if name != "stem":
                shapes[(Cin, Cout, R, st, pd, H)] += 1
    tot = defaultdict(lambda: [0.0, 0.0])
    print(f"{'pass':6s} {'Cin,Cout,R,s,p,H':26s} {'n':>2s} {'pipe ms':>8s} {'dma ms':>8s} {'ratio':>6s}",
          flush=True)
    for key, mult in sorted(shapes.items()):
        Cin, Cout, R, st, pd, H = key
        Ho = ops.out_hw(H, R, st, pd)
        x = torch.randn(G, B, H, H, Cin, device=dev).to(dt)
        w = (torch.randn(G, Cout, R, R, Cin, device=dev) * 0.05).to(dt)
        y = torch.empty(G, B, Ho, Ho, Cout, device=dev, dtype=dt)
        nblk = ops.fwd_stat_blocks(G, B, H, H, Cin, Cout, R, st, pd)
        stats = (torch.empty(G, nblk, Cout, device=dev), torch.empty(G, nblk, Cout, device=dev),
                 torch.empty(G, nblk, device=dev))
        xbn = (torch.rand(G, Cin, device=dev) + 0.5, torch.randn(G, Cin, device=dev), 1)
        dx = torch.empty_like(x)
        wt = torch.empty(G, R * R, Cin, Cout, device=dev, dtype=dt)
        ops.weights_rsck(w, G, Cout, R * R, Cin, wt)
        runs = {
            "fwd": (lambda: ops.conv2d_fwd(x, w, y, G, B, H, H, Cin, Cout, R, st, pd, stats=stats),
                    1),
            "fwdbn": (lambda: ops.conv2d_fwd(x, w, y, G, B, H, H, Cin, Cout, R, st, pd, x_bn=xbn,
                                             stats=stats), 2),
        }
        for p in a.passes.split(","):
            if p == "dgrad":
                if Cout % 32:
                    continue
                f0 = lambda: ops.conv2d_bwd_data(y, w, dx, G, B, H, H, Cin, Cout, R, st, pd)
                f1 = lambda: ops.conv2d_bwd_data(y, w, dx, G, B, H, H, Cin, Cout, R, st, pd,
                                                 w_rsck=wt)
                t0 = min(timeit(f0, a.reps) for _ in range(a.rounds))
                t1 = min(timeit(f1, a.reps) for _ in range(a.rounds))
                tr = timeit(lambda: ops.weights_rsck(w, G, Cout, R * R, Cin, wt), a.reps)
                t1 += tr
            else:
                fn, mode = runs[p]
                t0 = t1 = float("inf")
                for _ in range(a.rounds):
                    ops.set_dma16(0)
                    t0 = min(t0, timeit(fn, a.reps))
                    ops.set_dma16(mode)
                    t1 = min(t1, timeit(fn, a.reps))
                ops.set_dma16(1)
            tot[p][0] += t0 * mult
            tot[p][1] += t1 * mult
            print(f"{p:6s} {str(key):26s} {mult:2d} {t0:8.3f} {t1:8.3f} {t1 / t0:6.3f}", flush=True)
        del x, w, y, dx, wt
        torch.cuda.empty_cache()
    for p, (t0, t1) in tot.items():
        print(f"TOTAL {p:6s} pipe {t0:8.2f} ms  dma {t1:8.2f} ms  ratio {t1 / t0:.3f}", flush=True)


if __name__ == "__main__":
    main()
