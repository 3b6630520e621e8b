"""A/B of the BatchNorm-backward fold, interleaved in one
process: for every data-gradient shape of the bf16 training slice (G=5, B=64, 224 / 256 px)
whose dy is the backward of a ReLU BatchNorm,

  current: bn_bwd (partial sums + finalize + apply -> dy, 16-bit) ; dgrad(dy)
  fold   : bn_bwd partial sums + finalize only ; dgrad with dy = alpha*dz + beta*y + gamma
           computed in the A-loader from (y, dout)

The weight gradient also reads dy; the fold only pays if the dgrad's extra loader work costs
less than HALF the apply pass it removes (the WGRAD A-loader would pay the same again).

    python tools/fold_ab.py [--dtype bf16] [--rounds 3]
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
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    G, B, dev = a.G, a.B, "cuda"
    shapes = defaultdict(int)
    for cin, S in ((3, 224), (3, 256), (1, 256)):
        for name, Cin, Cout, R, st, pd, H in trunk_convs(cin, S):
            if name != "stem" and Cout % 64 == 0:
                shapes[(Cin, Cout, R, st, pd, H)] += 1
    tot = [0.0, 0.0, 0.0, 0.0]
    print(f"{'Cin,Cout,R,s,p,H':26s} {'n':>2s} {'apply':>7s} {'dgrad':>7s} {'dgrad+fold':>10s} "
          f"{'cur':>7s} {'fold':>7s}", flush=True)
    for key, mult in sorted(shapes.items()):
        Cin, Cout, R, st, pd, H = key
        Ho = ops.out_hw(H, R, st, pd)
        M = B * Ho * Ho
        w = (torch.randn(G, Cout, R, R, Cin, device=dev) * 0.05).to(dt)
        y = torch.randn(G, B, Ho, Ho, Cout, device=dev).to(dt)
        dout = torch.randn(G, B, Ho, Ho, Cout, device=dev).to(dt)
        dy = torch.empty_like(dout)
        dx = torch.empty(G, B, H, H, Cin, device=dev, dtype=dt)
        mean = torch.randn(G, Cout, device=dev) * 0.1
        invstd = torch.rand(G, Cout, device=dev) + 0.5
        sc = torch.rand(G, Cout, device=dev) + 0.5
        sh = torch.randn(G, Cout, device=dev) * 0.1
        ws = torch.empty(ops.bn_workspace_floats(G, M, Cout), device=dev)
        coef = torch.randn(5, G, Cout, device=dev)
        coef[3], coef[4] = sc, sh

        def apply_full():
            ops.bn_bwd(y, None, dout, 1, mean, invstd, sc, G, M, Cout, ws, dy, shift=sh)

        def partial_only():
            ops.bn_bwd(y, None, dout, 1, mean, invstd, sc, G, M, Cout, ws, None, shift=sh)

        def dgrad():
            ops.conv2d_bwd_data(dy, w, dx, G, B, H, H, Cin, Cout, R, st, pd)

        def dgrad_fold():
            ops.conv2d_bwd_data_fold(dout, y, coef, 1, w, dx, G, B, H, H, Cin, Cout, R, st, pd)

        t = {k: float("inf") for k in ("full", "part", "dg", "fold")}
        for _ in range(a.rounds):
            t["full"] = min(t["full"], timeit(apply_full, a.reps))
            t["part"] = min(t["part"], timeit(partial_only, a.reps))
            t["dg"] = min(t["dg"], timeit(dgrad, a.reps))
            t["fold"] = min(t["fold"], timeit(dgrad_fold, a.reps))
        apply = t["full"] - t["part"]
        cur, fold = t["full"] + t["dg"], t["part"] + t["fold"]
        tot[0] += mult * apply
        tot[1] += mult * t["dg"]
        tot[2] += mult * t["fold"]
        tot[3] += mult * (cur - fold)
        print(f"{str(key):26s} {mult:2d} {apply:7.3f} {t['dg']:7.3f} {t['fold']:10.3f} "
              f"{cur:7.3f} {fold:7.3f}", flush=True)
        del w, y, dout, dy, dx, ws
        torch.cuda.empty_cache()
    print(f"TOTAL apply pass {tot[0]:.2f} ms; dgrad {tot[1]:.2f} -> folded {tot[2]:.2f} ms "
          f"(+{tot[2] - tot[1]:.2f}); current - fold (dgrad side only) {tot[3]:+.2f} ms; the full "
          f"fold also pays the WGRAD loader (~+{tot[2] - tot[1]:.2f} ms): net "
          f"{tot[3] - (tot[2] - tot[1]):+.2f} ms", flush=True)


if __name__ == "__main__":
    main()
