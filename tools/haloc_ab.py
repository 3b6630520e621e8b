"""A/B of the chunked LDS row-image 16-bit 3x3 forwards (conv_haloc16.hip)
against the implicit GEMM (conv_pipe16 / conv_big16 routing, mauv_set_haloc16(0)) over every
3x3 / stride-1 forward of the three trunks over 128-512 channels (the bottleneck conv2s, pending
bn1 + ReLU on load), interleaved rounds in one process, max |difference| of the outputs printed
(the two sum in different orders).

    python tools/haloc_ab.py [--dtype bf16|f16] [--G 5] [--B 64] [--rounds 3]
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--arms", default="0,1,2", help="mauv_set_haloc16 modes to compare "
                    "(0: the implicit GEMM, 1 / 2: conv_haloc16 with 32 x 64 / 64 x 64 wave tiles)")
    a = ap.parse_args()
    ARMS = [int(v) for v in a.arms.split(",")]
    dt = {"bf16": torch.bfloat16, "f16": torch.float16}[a.dtype]
    G, B = a.G, a.B
    torch.manual_seed(0)
    shapes = {}
    for trunk, cin, S in (("opt", 3, 224), ("bathy", 3, 256), ("sss", 1, 256)):
        for name, Cin, Cout, R, st, pd, H in trunk_convs(cin, S):
            if R == 3 and st == 1 and Cin in (128, 256, 512):
                shapes.setdefault((Cin, Cout, H, True), []).append(f"{trunk}:{name}")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {k: {arm: [] for arm in ARMS} for k in shapes}
    for rnd in range(a.rounds):
        for key in shapes:
            Cin, Cout, H, xb = key
            x = torch.randn(G, B, H, H, Cin, device="cuda").to(dt)
            w = (torch.randn(G, Cout, 3, 3, Cin, device="cuda") / (9 * Cin) ** 0.5).to(dt)
            nblk = ops.fwd_stat_blocks(G, B, H, H, Cin, Cout, 3, 1, 1)
            stats = tuple(torch.empty(*s, device="cuda") for s in ((G, nblk, Cout), (G, nblk, Cout),
                                                                  (G, nblk)))
            x_bn = (torch.rand(G, Cin, device="cuda") + 0.5,
                    torch.randn(G, Cin, device="cuda") * 0.1, 1) if xb else None
            outs = {}
            for arm in (ARMS if rnd % 2 == 0 else ARMS[::-1]):
                y = torch.empty(G, B, H, H, Cout, device="cuda", dtype=dt)
                prev = ops.set_haloc16(arm)
                try:
                    fn = lambda: ops.conv2d_fwd(x, w, y, G, B, H, H, Cin, Cout, 3, 1, 1,
                                                x_bn=x_bn, stats=stats)
                    fn()
                    e0.record()
                    for _ in range(a.reps):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                finally:
                    ops.set_haloc16(prev)
                res[key][arm].append(e0.elapsed_time(e1) / a.reps)
                outs[arm] = y
            if rnd == 0:
                d = max((outs[ARMS[0]].float() - outs[arm].float()).abs().max().item() for arm in ARMS)
                print(f"{key} max|diff| {d:.3g} of max|y| {outs[ARMS[0]].float().abs().max().item():.3g}",
                      flush=True)
            del x, w, outs
    tot = {arm: 0.0 for arm in ARMS}
    print(f"{'Cin,Cout,H,xbn':22s} {'n':>3s} " + " ".join(f"{'ms@' + str(x):>9s}" for x in ARMS) +
          " " + " ".join(f"{'GB/s@' + str(x):>9s}" for x in ARMS) + "  layers")
    for key, v in sorted(shapes.items(), key=lambda kv: -min(res[kv[0]][ARMS[0]])):
        Cin, Cout, H, xb = key
        nb = 2 * G * (B * H * H * (Cin + Cout) + 9 * Cin * Cout)
        t = {arm: min(res[key][arm]) for arm in ARMS}
        for arm in ARMS:
            tot[arm] += t[arm] * len(v)
        print(f"{str(key):22s} {len(v):3d} " + " ".join(f"{t[x]:9.3f}" for x in ARMS) + " " +
              " ".join(f"{nb / t[x] / 1e6:9.0f}" for x in ARMS) + f"  {' '.join(v[:4])}")
    print("TOTAL (x occurrences): " + ", ".join(f"mode {x} {tot[x]:.2f} ms" for x in ARMS))


if __name__ == "__main__":
    main()
