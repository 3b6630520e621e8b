"""A/B of the block-output fold (engine.FOLD; ops.conv2d_fwd_fold) on the
bench's f16 MC-inference workload (B=256, N=100, 224 / 256 px, mc_statistics under autocast
like the drop-in predictor): interleaved rounds in one process, HIP-event-free wall clock of
whole batches after a warm-up chunk.

    python tools/fold_ab.py [--rounds 3] [--batch 256] [--mc 100] [--sonar 256]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from mauv import engine  # noqa: E402
from mauv.predict import mc_statistics, mc_chunk  # noqa: E402
from mauv.models import define_models, DEFAULT_PRIOR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--mc", type=int, default=100)
    ap.add_argument("--sonar", type=int, default=256)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = define_models(None, 7, DEFAULT_PRIOR)["multimodal_model"].to(dev)
    x, b, s, _ = bench.synthetic_batch(a.batch, 224, a.sonar, dev, 99)
    hw = [(224, 224), (a.sonar, a.sonar), (a.sonar, a.sonar)]
    chunk = mc_chunk(model, a.batch, a.mc, dtype=torch.float16, device=dev, hw=hw)
    res = {False: [], True: []}
    outs = {}
    for r in range(a.rounds):
        for fold in ((False, True) if r % 2 == 0 else (True, False)):
            engine.FOLD = fold
            with torch.no_grad(), torch.autocast("cuda"):
                mc_statistics(model, x, b, s, chunk, chunk=chunk)   # warm-up chunk
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                o = mc_statistics(model, x, b, s, a.mc, chunk=chunk)
                torch.cuda.synchronize()
                res[fold].append(time.perf_counter() - t0)
            outs[fold] = o
            print(f"round {r} fold={int(fold)}: {a.mc * a.batch / res[fold][-1]:.0f} "
                  f"MC-samples/s ({res[fold][-1] * 1e3:.0f} ms)", flush=True)
    engine.FOLD = True
    for f in (False, True):
        t = min(res[f])
        print(f"fold={int(f)} best {a.mc * a.batch / t:.0f} MC-samples/s ({t * 1e3:.0f} ms), "
              f"mc_chunk {chunk}")
    print(f"speedup {min(res[False]) / min(res[True]):.3f}x")


if __name__ == "__main__":
    main()
