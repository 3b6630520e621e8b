"""Per-shape timing of the implicit-GEMM conv kernels at the bench workload (G=5 MC groups,
B=64, 224 optical / 256 sonar trunks).  Prints TF/s per (trunk, layer, pass) and totals.

    python tools/conv_bench.py [--G 5] [--B 64] [--only fwd,dgrad,wgrad] [--top 20]
"""
import argparse
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd")]
import torch  # noqa: E402
from mauv import ops  # noqa: E402


def trunk_convs(cin, S):
    """(name, Cin, Cout, R, stride, pad, H) for every conv of a ResNet-50 trunk."""
    out = [("stem", cin, 64, 7, 2, 3, S)]
    H = (S + 6 - 7) // 2 + 1
    H = (H + 2 - 3) // 2 + 1
    inp = 64
    for li, (planes, blocks, st) in enumerate(((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2))):
        for bi in range(blocks):
            s = st if bi == 0 else 1
            out.append((f"l{li+1}.{bi}.c1", inp, planes, 1, 1, 0, H))
            out.append((f"l{li+1}.{bi}.c2", planes, planes, 3, s, 1, H))
            H2 = (H + 2 - 3) // s + 1
            out.append((f"l{li+1}.{bi}.c3", planes, planes * 4, 1, 1, 0, H2))
            if bi == 0:
                out.append((f"l{li+1}.{bi}.ds", inp, planes * 4, 1, s, 0, H))
            inp = planes * 4
            H = H2
    return out


REPS = 5


def timeit(fn, reps=None):
    reps = reps or REPS
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
    ap.add_argument("--G", type=int, default=5)
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--only", default="fwd,dgrad,wgrad")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--trunks", default="opt,bathy,sss")
    ap.add_argument("--shape", default="", help="one shape Cin,Cout,R,stride,pad,H (profiling)")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16", "f16"])
    ap.add_argument("--xpad", type=int, default=0,
                    help="FWD: store x with a row pitch of Cin + xpad channels (strided loads)")
    ap.add_argument("--mark", action="store_true",
                    help="launch a torch.flip marker kernel before each timed pass and print "
                         "'MARK' lines (per-shape PMC traffic: tools/shape_traffic.py)")
    ap.add_argument("--fused", action="store_true",
                    help="as in the model: BN+ReLU applied on load (fwd, wgrad) and BN "
                         "statistics partials from the fwd epilogue")
    ap.add_argument("--haloc16", type=int, default=None,
                    help="mauv_set_haloc16 mode for the run (0: the implicit GEMM)")
    ap.add_argument("--expand16", type=int, default=None,
                    help="mauv_set_expand16 mode for the run (0: the implicit GEMM)")
    a = ap.parse_args()
    if a.expand16 is not None:
        ops.set_expand16(a.expand16)
    if a.haloc16 is not None:
        ops.set_haloc16(a.haloc16)
    global REPS
    REPS = a.reps
    G, B, dev = a.G, a.B, "cuda"
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}[a.dtype]
    kinds = a.only.split(",")
    rows = []
    cache = {}
    marker = torch.zeros(2, device=dev)
    nmark = [0]

    def mark(trunk, name, kind, key, nbytes):
        if a.mark:
            torch.cuda.synchronize()
            torch.flip(marker, [0])
            torch.cuda.synchronize()
            print(f"MARK {nmark[0]} {trunk} {name} {kind} {','.join(map(str, key))} {nbytes} "
                  f"{REPS + 1}", flush=True)
            nmark[0] += 1
    for trunk, cin, S in (("opt", 3, 224), ("bathy", 3, 256), ("sss", 1, 256)):
        if trunk not in a.trunks:
            continue
        convs = trunk_convs(cin, S)
        if a.shape:
            convs = [("shape",) + tuple(int(v) for v in a.shape.split(","))]
        for name, Cin, Cout, R, st, pd, H in convs:
            key = (Cin, Cout, R, st, pd, H)
            Ho = ops.out_hw(H, R, st, pd)
            fl = 2.0 * G * B * Ho * Ho * Cout * R * R * Cin
            esz = 4 if a.dtype == "fp32" else 2
            # algorithmic HBM bytes of one launch: each operand read once, the output written once
            # (wgrad: its fp32 split-K slabs are written once)
            nx, ny, nw = G * B * H * H * Cin, G * B * Ho * Ho * Cout, G * Cout * R * R * Cin
            sp_ = ops.wgrad_splits(G, B, H, H, Cin, Cout, R, st, pd)
            byt = {"fwd": esz * (nx + nw + ny), "dgrad": esz * (ny + nw + nx),
                   "wgrad": esz * (nx + ny) + 4 * sp_ * nw}
            if key in cache:
                for kind, ms in cache[key]:
                    rows.append((trunk, name, kind, key, ms, fl, byt[kind]))
                continue
            res = []
            if dt != torch.float32 and Cin % 8:
                Cin = 8   # the 16-bit path zero-pads the stems' input channels to 8
            xfull = torch.randn(G, B, H, H, Cin + a.xpad, device=dev).to(dt)
            x = xfull[..., :Cin] if a.xpad else xfull
            xstr = None
            if a.xpad:
                P = Cin + a.xpad
                xstr = (B * H * H * P, H * H * P, H * P, P, 1)
            w = (torch.randn(G, Cout, R, R, Cin, device=dev) * 0.05).to(dt)
            y = torch.empty(G, B, Ho, Ho, Cout, device=dev, dtype=dt)
            xbn, stats = None, None
            if a.fused and name != "stem":
                xbn = (torch.rand(G, Cin, device=dev) + 0.5, torch.randn(G, Cin, device=dev), 1)
                nblk = ops.fwd_stat_blocks(G, B, H, H, Cin, Cout, R, st, pd)
                stats = (torch.empty(G, nblk, Cout, device=dev), torch.empty(G, nblk, Cout, device=dev),
                         torch.empty(G, nblk, device=dev))
            if "fwd" in kinds:
                mark(trunk, name, "fwd", key, byt["fwd"])
                res.append(("fwd", timeit(lambda: ops.conv2d_fwd(xfull if a.xpad else x, w, y, G, B, H, H, Cin, Cout, R, st, pd,
                                                                 x_bn=xbn, stats=stats,
                                                                 x_strides=xstr))))
            if "dgrad" in kinds and name != "stem" and (dt == torch.float32 or Cout % 32 == 0):
                dx = torch.empty_like(x)
                mark(trunk, name, "dgrad", key, byt["dgrad"])
                res.append(("dgrad", timeit(lambda: ops.conv2d_bwd_data(y, w, dx, G, B, H, H, Cin, Cout, R, st, pd))))
                del dx
            if "wgrad" in kinds:
                sp = ops.wgrad_splits(G, B, H, H, Cin, Cout, R, st, pd)
                ws = torch.empty(sp, G, Cout, R * R * Cin, device=dev)
                mark(trunk, name, "wgrad", key, byt["wgrad"])
                res.append(("wgrad", timeit(lambda: ops.conv2d_bwd_weight(x, y, ws, sp, G, B, H, H, Cin, Cout, R, st, pd,
                                                                          x_bn=xbn))))
                del ws
            del x, w, y
            torch.cuda.empty_cache()
            cache[key] = res
            for kind, ms in res:
                rows.append((trunk, name, kind, key, ms, fl, byt[kind]))
    # per-launch roofline time: max(flops / MFMA peak, algorithmic bytes / HBM peak)
    peak = 2.5e15 / 6 if a.dtype == "fp32" else 2.5e15
    tot = defaultdict(lambda: [0.0, 0.0, 0.0])
    for r in rows:
        tot[r[2]][0] += r[4]
        tot[r[2]][1] += r[5]
        tot[r[2]][2] += max(r[5] / peak, r[6] / 8e12) * 1e3
    print(f"{'trunk':6s} {'layer':10s} {'pass':6s} {'Cin,Cout,R,s,p,H':28s} {'ms':>8s} {'TF/s':>7s} {'GB/s':>7s} {'roof':>5s}")
    for r in sorted(rows, key=lambda r: -r[4])[:a.top]:
        rt = max(r[5] / peak, r[6] / 8e12) * 1e3
        print(f"{r[0]:6s} {r[1]:10s} {r[2]:6s} {str(r[3]):28s} {r[4]:8.3f} {r[5] / r[4] / 1e9:7.1f} "
              f"{r[6] / r[4] / 1e6:7.0f} {rt / r[4]:5.2f}")
    for k, (ms, fl, rt) in tot.items():
        print(f"TOTAL {k:6s}: {ms:8.2f} ms  {fl / 1e12:8.2f} TFLOP  {fl / ms / 1e9:6.1f} TF/s  "
              f"roofline {rt:7.2f} ms ({rt / ms:.2f})")
    allms = sum(v[0] for v in tot.values())
    allfl = sum(v[1] for v in tot.values())
    print(f"TOTAL all   : {allms:8.2f} ms  {allfl / allms / 1e9:6.1f} TF/s")


if __name__ == "__main__":
    main()
