"""Probe driver (not product code): the LDS-DMA big-tile grouped GEMM (gemm_glds.hip) against
torch.bmm (hipBLASLt) and the product 16-bit 1x1-conv forward (conv_pipe16) on the trunks' 1x1
shapes at the bench workload (G = 5 MC groups, B = 64).  Checks each result against fp32 torch,
then times interleaved rounds with HIP events.

    make -C tools/probe && python tools/probe/run_probe.py
"""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-auv_amd")]

from mauv import ops  # noqa: E402

lib = ctypes.CDLL(os.path.join(HERE, "libprobe.so"))
lib.probe_gemm_glds.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int] * 4 + \
    [ctypes.c_void_p] * 3

# (name, M per group, N, K): 1x1 convs of the bench trunks (B = 64; sonar 256 px / optical 224)
SHAPES = [
    ("l4 c1 2048->512 @8", 64 * 64, 512, 2048),
    ("l4 c3 512->2048 @8", 64 * 64, 2048, 512),
    ("l4.0 c1 1024->512 @16", 64 * 256, 512, 1024),
    ("l3 c1 1024->256 @16", 64 * 256, 256, 1024),
    ("l3 c3 256->1024 @16", 64 * 256, 1024, 256),
    ("l3.0 ds 512->1024 @16", 64 * 256, 1024, 512),
    ("l2 c1 512->128 @32", 64 * 1024, 128, 512),
    ("square 16k x 1k x 1k", 16384, 1024, 1024),
]
G = 5
TRACE = os.environ.get("PROBE_TRACE") == "1"
VARIANTS = {0: "glds 256x256", 1: "glds 256x128", 2: "glds 256x128 x3", 3: "glds 128x128"}
XVARIANTS = {4: "glds 256x128 +BN", 5: "glds 256x256 +BN"}


def ev_time(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def main():
    torch.manual_seed(0)
    dt = torch.bfloat16
    stream = torch.cuda.current_stream().cuda_stream
    for xbn in (False, True):
        vs = XVARIANTS if xbn else VARIANTS
        print(("pending BN + ReLU on A (XBN)" if xbn else "plain A") + ":")
        print(f"{'shape':26s} {'GFLOP':>7s} " + " ".join(f"{v:>16s}" for v in
              ["torch.bmm", "conv_pipe16", "conv_big16"] + list(vs.values())))
        for name, M, N, K in SHAPES:
            run_shape(name, M, N, K, xbn, vs, dt, stream)


def run_shape(name, M, N, K, xbn, vs, dt, stream):
    A = (torch.rand(G, M, K, device="cuda") * 2 - 1).to(dt)
    B = (torch.rand(G, N, K, device="cuda") * 2 - 1).to(dt)
    sc = torch.rand(G, K, device="cuda") + 0.5
    sh = torch.rand(G, K, device="cuda") - 0.5
    Ar = torch.relu(A.float() * sc[:, None, :] + sh[:, None, :]).to(dt).float() if xbn else A.float()
    ref = torch.bmm(Ar, B.float().transpose(1, 2))
    C = torch.empty(G, M, N, device="cuda", dtype=dt)
    fns = {"torch.bmm": lambda: torch.bmm(A, B.transpose(1, 2))}
    Hh = M // 64
    x_bn = (sc, sh, 1) if xbn else None
    def conv(big):
        prev = ops.set_big16(big, 64)
        try:
            ops.conv2d_fwd(A, B, C, G, 64, Hh, 1, K, N, 1, 1, 0, x_bn=x_bn)
        finally:
            ops.set_big16(prev)
    fns["conv_pipe16"] = lambda: conv(False)
    fns["conv_big16"] = lambda: conv(True)
    for v in vs:
        fns[vs[v]] = (lambda v=v: lib.probe_gemm_glds(v, A.data_ptr(), B.data_ptr(),
                                                      C.data_ptr(), M, N, K, G, sc.data_ptr(),
                                                      sh.data_ptr(), stream))
    errs = {}
    for k, f in fns.items():
        C.zero_()
        torch.cuda.synchronize()
        if TRACE:   # which launch faults (gpurun_out/probe1.log's shape 3): one line per launch
            print(f"  [trace] {name} {'XBN ' if xbn else ''}{k}: launch", flush=True)
        out = f()
        torch.cuda.synchronize()
        if TRACE:
            print(f"  [trace] {name} {k}: ok", flush=True)
        if isinstance(out, int) and out != 0:
            errs[k] = f"rc {out}"
            continue
        got = out if isinstance(out, torch.Tensor) else C
        r = ref if k != "torch.bmm" else torch.bmm(A.float(), B.float().transpose(1, 2))
        errs[k] = ((got.float() - r).abs().max() / r.abs().max()).item()
    times = {k: [] for k in fns}
    for _ in range(5):
        for k, f in fns.items():
            if isinstance(errs[k], str):
                continue
            times[k].append(ev_time(f, 10))
    fl = 2.0 * G * M * N * K
    cells = []
    for k in fns:
        if isinstance(errs[k], str) or errs[k] > 2e-2:
            cells.append(f"{'ERR ' + str(errs[k])[:10]:>16s}")
        else:
            t = sorted(times[k])[len(times[k]) // 2]
            cells.append(f"{t * 1e3:7.1f}us {fl / t / 1e9:5.0f}T")
    print(f"{name:26s} {fl / 1e9:7.1f} " + " ".join(cells), flush=True)

if __name__ == "__main__":
    main()
