"""Per-shape conv time INSIDE a training step (the bench's step: B=64, num_mc=5, trunks in
sequence so each launch's HIP-event duration is its own), grouped by (pass, shape, epilogue
form).  conv_bench.py times the bare kernels; this shows what the step's calls cost with their
addends / accumulation / pending BN (the fp32 data gradient's in-step rate).

    python tools/step_shapes.py [--dtype fp32|bf16] [--top 40]
"""
import argparse
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd")]
import torch  # noqa: E402

from bench import synthetic_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--num-mc", type=int, default=5)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    from mauv import ops, engine
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
    engine.TRUNK_STREAMS = False
    step()
    torch.cuda.synchronize()
    ops.PROFILE, ops.PROFILE_INFO = [], []
    step()
    torch.cuda.synchronize()
    rows, info = ops.PROFILE, ops.PROFILE_INFO
    ops.PROFILE = ops.PROFILE_INFO = None
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    kinds = collections.defaultdict(lambda: [0.0, 0.0])
    for (kind, fl, nb, nl, e0, e1), inf in zip(rows, info):
        ms = e0.elapsed_time(e1)
        d = agg[(kind, inf)]
        d[0] += 1
        d[1] += ms
        d[2] += fl
        d[3] += nb
        kinds[kind][0] += ms
        kinds[kind][1] += fl
    print(f"{'pass':14s} {'shape (G,B,H,W,Cin,Cout,R,s,p,extra)':58s} {'n':>3s} {'ms':>8s} "
          f"{'ms/call':>8s} {'TF/s':>7s} {'GB/s':>7s}")
    for (kind, inf), (n, ms, fl, nb) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{kind:14s} {str(inf):58s} {n:3d} {ms:8.3f} {ms / n:8.3f} "
              f"{fl / ms / 1e9:7.1f} {nb / ms / 1e6:7.0f}")
    for k, (ms, fl) in sorted(kinds.items()):
        print(f"TOTAL {k:14s} {ms:8.2f} ms  {fl / ms / 1e9:7.1f} TF/s")


if __name__ == "__main__":
    main()
