"""The block-output fold (conv_big16 RES) per shape: every identity block's
conv1 of the three trunks (Cin = 4 planes -> planes, the previous block output formed on load),
timed alone at an f16 inference chunk (default G = 20, B = 256) with its algorithmic HBM rate,
beside the unfused pair it replaces (bn_apply_mask into the block output, then the plain conv1).

    python tools/fold_bench.py [--dtype f16|bf16] [--G 20] [--B 256] [--reps 3] [--shape Cin,Cout,H]
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
    ap.add_argument("--dtype", default="f16", choices=["bf16", "f16"])
    ap.add_argument("--G", type=int, default=20)
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--shape", default="", help="one shape Cin,Cout,H (profiling)")
    ap.add_argument("--only-fold", action="store_true", help="time the fold alone (PMC runs)")
    a = ap.parse_args()
    dt = {"bf16": torch.bfloat16, "f16": torch.float16}[a.dtype]
    G, B, dev = a.G, a.B, "cuda"
    shapes = {}
    for trunk, cin, S in (("opt", 3, 224), ("bathy", 3, 256), ("sss", 1, 256)):
        for name, Cin, Cout, R, st, pd, H in trunk_convs(cin, S):
            if name.endswith("c1") and not name.endswith(".0.c1"):
                shapes.setdefault((Cin, Cout, H), []).append(f"{trunk}:{name}")
    if a.shape:
        shapes = {tuple(int(v) for v in a.shape.split(",")): ["shape"]}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    print(f"{'Cin,Cout,H':16s} {'n':>3s} {'fold ms':>9s} {'GB/s':>7s} {'pair ms':>9s}  layers")
    tot = [0.0, 0.0]
    for (Cin, Cout, H), v in sorted(shapes.items()):
        M = B * H * H
        y3 = torch.randn(G, B, H, H, Cin, device=dev).to(dt)
        res = torch.randn(G, B, H, H, Cin, device=dev).to(dt)
        sc = torch.rand(G, Cin, device=dev) + 0.5
        sh = torch.randn(G, Cin, device=dev) * 0.1
        out = torch.empty_like(y3)
        mask = torch.empty(G * M * Cin // 8, dtype=torch.uint8, device=dev)
        w = (torch.randn(G, Cout, 1, 1, Cin, device=dev) / Cin ** 0.5).to(dt)
        y1 = torch.empty(G, B, H, H, Cout, device=dev, dtype=dt)
        nblk = ops.fwd_stat_blocks(G, B, H, H, Cin, Cout, 1, 1, 0)
        stats = tuple(torch.empty(*s, device=dev) for s in ((G, nblk, Cout), (G, nblk, Cout), (G, nblk)))

        def fold():
            assert ops.conv2d_fwd_fold(y3, sc, sh, res, None, out, w, y1, G, B, H, H, Cin, Cout,
                                       stats=stats, mask=mask)

        def pair():
            ops.bn_apply_mask(y3, sc, sh, res, out, mask, G, M, Cin)
            ops.conv2d_fwd(out, w, y1, G, B, H, H, Cin, Cout, 1, 1, 0, stats=stats)
        t = []
        for fn in ((fold,) if a.only_fold else (fold, pair)):
            fn()
            e0.record()
            for _ in range(a.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            t.append(e0.elapsed_time(e1) / a.reps)
        nb = 2 * G * (3 * M * Cin + M * Cout + Cout * Cin)
        tot[0] += t[0] * len(v)
        t.append(float("nan"))
        tot[1] += t[1] * len(v)
        print(f"{str((Cin, Cout, H)):16s} {len(v):3d} {t[0]:9.3f} {nb / t[0] / 1e6:7.0f} {t[1]:9.3f}  "
              f"{' '.join(v[:4])}", flush=True)
        del y3, res, out, mask, y1
        torch.cuda.empty_cache()
    print(f"TOTAL (x occurrences): fold {tot[0]:.2f} ms, unfused pair {tot[1]:.2f} ms")


if __name__ == "__main__":
    main()
