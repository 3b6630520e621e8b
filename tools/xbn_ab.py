"""The pending BN(+ReLU) applied on load (x_bn) against materialising it first: every 16-bit
forward of the three trunks whose input is a lazily applied BN (conv2, conv3), timed three ways
in interleaved rounds — (a) the conv with x_bn; (b) bn_apply into a tensor, then the conv
without x_bn; (c) the conv without x_bn alone (what (b) pays beyond the pass).

    python tools/xbn_ab.py [--dtype f16|bf16] [--G 20] [--B 256] [--rounds 3]
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dt = {"bf16": torch.bfloat16, "f16": torch.float16}[a.dtype]
    G, B, dev = a.G, a.B, "cuda"
    torch.manual_seed(0)
    shapes = {}
    for trunk, cin, S in (("opt", 3, 224), ("bathy", 3, 256), ("sss", 1, 256)):
        for name, Cin, Cout, R, st, pd, H in trunk_convs(cin, S):
            if not name.endswith(("c2", "c3")):
                continue
            shapes.setdefault((Cin, Cout, R, st, pd, H), []).append(f"{trunk}:{name}")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {k: {m: [] for m in "abc"} for k in shapes}

    def timed(fn):
        fn()
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    for rnd in range(a.rounds):
        for key in shapes:
            Cin, Cout, R, st, pd, H = key
            Ho = ops.out_hw(H, R, st, pd)
            x = torch.randn(G, B, H, H, Cin, device=dev).to(dt)
            xm = torch.empty_like(x)
            w = (torch.randn(G, Cout, R, R, Cin, device=dev) * 0.05).to(dt)
            y = torch.empty(G, B, Ho, Ho, Cout, device=dev, dtype=dt)
            nblk = ops.fwd_stat_blocks(G, B, H, H, Cin, Cout, R, st, pd)
            stats = tuple(torch.empty(*s, device=dev) for s in ((G, nblk, Cout), (G, nblk, Cout),
                                                               (G, nblk)))
            sc, sh = torch.rand(G, Cin, device=dev) + 0.5, torch.randn(G, Cin, device=dev) * 0.1
            fa = lambda: ops.conv2d_fwd(x, w, y, G, B, H, H, Cin, Cout, R, st, pd,
                                        x_bn=(sc, sh, 1), stats=stats)
            fc = lambda: ops.conv2d_fwd(xm, w, y, G, B, H, H, Cin, Cout, R, st, pd, stats=stats)

            def fb():
                ops.bn_apply(x, sc, sh, None, 1, xm, G, B * H * H, Cin)
                fc()
            for m, fn in (("a", fa), ("b", fb), ("c", fc)):
                res[key][m].append(timed(fn))
            del x, xm, w, y
    tot = {m: 0.0 for m in "abc"}
    print(f"{'Cin,Cout,R,s,H':24s} {'n':>3s} {'x_bn ms':>8s} {'pass+conv':>9s} {'conv':>8s}  layers")
    for key, v in sorted(shapes.items(), key=lambda kv: -min(res[kv[0]]["a"])):
        t = {m: min(res[key][m]) for m in "abc"}
        for m in "abc":
            tot[m] += t[m] * len(v)
        print(f"{str(key[:4] + key[5:]):24s} {len(v):3d} {t['a']:8.3f} {t['b']:9.3f} {t['c']:8.3f}  "
              f"{' '.join(v[:4])}")
    print(f"TOTAL (x occurrences): x_bn {tot['a']:.2f} ms, pass+conv {tot['b']:.2f} ms, "
          f"conv alone {tot['c']:.2f} ms")


if __name__ == "__main__":
    main()
