"""Which host calls launch torch's own fill / copy kernels during a training step (VERDICT r4
next 7: ~467 FillFunctor and ~281 copyBuffer launches per bf16 step).  One warm step, then one
step under torch.profiler with Python stacks; prints the aten::fill_ / zero_ / copy_ / to ops
grouped by the innermost mauv frame.

    python tools/host_ops.py [--dtype bf16|fp32] [--batch 64]
"""
import argparse
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd")]
import torch  # noqa: E402
from torch.profiler import profile, ProfilerActivity  # noqa: E402

from bench import synthetic_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--num-mc", type=int, default=5)
    a = ap.parse_args()
    from mauv.models import define_models, DEFAULT_PRIOR
    from mauv.train import mc_train_step
    from mauv.optim import FusedAdam
    from mauv.engine import set_precision
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = define_models(None, 7, DEFAULT_PRIOR)["multimodal_model"].to(dev)
    if a.dtype == "bf16":
        set_precision(model, torch.bfloat16)
    opt = FusedAdam(model.parameters(), lr=5e-5)
    crit = torch.nn.CrossEntropyLoss()
    x, b, s, y = synthetic_batch(a.batch, 224, 256, dev, 1)

    def step():
        return mc_train_step(model, (x, b, s), y, crit, opt, a.num_mc, a.batch, 2.0 ** -29)
    step()
    step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    want = ("aten::fill_", "aten::zero_", "aten::copy_", "aten::_to_copy", "aten::zeros",
            "aten::zeros_like", "aten::full", "aten::clone")
    by = collections.Counter()
    for ev in prof.events():
        if ev.name not in want or ev.device_type != torch.autograd.DeviceType.CPU:
            continue
        frames = [f for f in (ev.stack or []) if "mauv" in f or "bench" in f or "torch/" not in f]
        site = frames[0] if frames else (ev.stack[0] if ev.stack else "?")
        by[(ev.name, site)] += 1
    kern = collections.Counter()
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA and (
                "Fill" in ev.name or "copyBuffer" in ev.name or "Memcpy" in ev.name or
                "Memset" in ev.name):
            kern[ev.name[:90]] += 1
    print(f"device fill / copy launches in one {a.dtype} step:")
    for k, n in kern.most_common():
        print(f"  {n:5d}  {k}")
    print("host ops by call site:")
    for (name, site), n in by.most_common(40):
        print(f"  {n:5d}  {name:16s} {site}")


if __name__ == "__main__":
    main()
