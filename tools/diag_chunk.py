"""MC inference throughput vs MC chunk size (f16 autocast, B=256, N=100)."""
import os
import sys
import time

import torch

R = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "multimodal-auv_amd"))
import bench  # noqa: E402
from mauv.models import define_models, DEFAULT_PRIOR  # noqa: E402
from mauv.predict import mc_statistics  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
model = define_models(None, 7, DEFAULT_PRIOR)["multimodal_model"].to(dev)
x, b, s, _ = bench.synthetic_batch(256, 224, 256, dev, 99)
for chunk in (20, 25, 34, 50, 20):
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        mc_statistics(model, x, b, s, 2 * chunk, chunk=chunk)   # warm-up
        torch.cuda.synchronize()
        t = time.perf_counter()
        mc_statistics(model, x, b, s, 100, chunk=chunk)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
    print(f"chunk {chunk}: {100 * 256 / dt:.0f} MC-samples/s, peak {torch.cuda.max_memory_allocated() / 2**30:.1f} GiB", flush=True)
