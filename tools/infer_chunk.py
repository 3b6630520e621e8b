"""MC inference throughput vs MC chunk size (samples per batched launch), bench workload."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from mauv.predict import mc_statistics  # noqa: E402
from mauv.models import define_models, DEFAULT_PRIOR  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = define_models(None, 7, DEFAULT_PRIOR)["multimodal_model"].to(dev)
    x, b, s, _ = bench.synthetic_batch(256, 224, 256, dev, 99)
    for chunk in [int(c) for c in sys.argv[1:]] or [15, 20, 25, 34]:
        with torch.no_grad(), torch.autocast("cuda"):
            mc_statistics(model, x, b, s, chunk, chunk=chunk)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            mc_statistics(model, x, b, s, 100, chunk=chunk)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        print(f"chunk {chunk}: {100 * 256 / dt:.0f} MC-samples/s ({dt * 1e3:.0f} ms)", flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
