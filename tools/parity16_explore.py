"""Where does torch-autocast's own 16-bit training step resolve the float64 gradient direction
of whole trunks?  (judge the whole-trunk cosines at such a shape.)  Prints
the whole-gradient cosines of HIP and torch-autocast against a float64 oracle run on the GPU.

    python tools/parity16_explore.py [--dtype bf16] S_opt,S_son,B,N ...
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd")]
import torch  # noqa: E402

from tests.test_parity16_gpu import train_step16_cosines  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16"])
    ap.add_argument("--fit", type=int, default=0, help="train the model this many fp32 steps first")
    ap.add_argument("shapes", nargs="+")
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    for sh in a.shapes:
        S_opt, S_son, B, N = (int(v) for v in sh.split(","))
        t0 = time.time()
        r = train_step16_cosines(dt, S_opt, S_son, B, N, truth_device="cuda", fp32_cpu=False,
                                 fit_steps=a.fit)
        cells = "  ".join(f"{g[:5]} HIP {c['hip']:.3f} ac {c['autocast']:.3f}"
                          for g, c in r["whole"].items())
        print(f"{a.dtype} fit={a.fit} {S_opt}/{S_son} B={B} N={N} ({time.time() - t0:.0f} s): {cells}  "
              f"dlogit HIP {r['dlogit_hip']:.2e} ac {r['dlogit_autocast']:.2e}", flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
