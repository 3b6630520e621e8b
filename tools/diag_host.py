"""Host enqueue time vs GPU time of the bench training step (is the step launch-bound?)."""
import os
import sys
import time

import torch

R = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "multimodal-auv_amd"))
import bench  # noqa: E402
from mauv.models import define_models, DEFAULT_PRIOR  # noqa: E402
from mauv.train import mc_loss, _grads_finite  # noqa: E402
from mauv.optim import FusedAdam  # noqa: E402
from mauv.engine import set_precision  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
model = define_models(None, 7, DEFAULT_PRIOR)["multimodal_model"].to(dev)
opt = FusedAdam(model.parameters(), lr=5e-5)
crit = torch.nn.CrossEntropyLoss()
x, b, s, y = bench.synthetic_batch(64, 224, 256, dev, 1)
for prec in (torch.bfloat16, None):
    set_precision(model, prec)
    for it in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loss, *_ = mc_loss(model, (x, b, s), y, crit, 5, 64, 1e-9)
        t1 = time.perf_counter()
        torch.isfinite(loss).item()
        t2 = time.perf_counter()
        loss.backward()
        t3 = time.perf_counter()
        ok = _grads_finite(model)
        t4 = time.perf_counter()
        opt.step()
        opt.zero_grad()
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        if it:
            print(prec, f"fwd enqueue {1e3*(t1-t0):.1f} ms, fwd done {1e3*(t2-t0):.1f}; "
                  f"bwd enqueue {1e3*(t3-t2):.1f}, bwd done {1e3*(t4-t2):.1f}; adam {1e3*(t5-t4):.1f}; "
                  f"step {1e3*(t5-t0):.1f}")
