"""A/B of the block-output fold (engine.FOLD; ops.conv2d_fwd_fold) on the
bench's f16 MC-inference workload (B=256, N=100, 224 / 256 px, mc_statistics under autocast
like the drop-in predictor) or, with --train, its bf16 training step (B=64, num_mc=5,
mc_train_step + FusedAdam): interleaved rounds in one process, wall clock of whole batches /
steps after warm-up.

    python tools/fold_ab.py [--rounds 3] [--batch 256] [--mc 100] [--sonar 256] [--only 0|1]
    python tools/fold_ab.py --train [--rounds 3] [--steps 10] [--dtype fp32] [--flag BWD_PARTIALS_F32]
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


def _set(flag, on):
    """An engine switch (engine.FOLD, ...) or a library routing switch named ops.set_<flag>
    (e.g. --flag expand16; --flag haloc16:3 sets mode 3 instead of 0 for the "off" arm)."""
    from mauv import ops
    name, _, off = flag.partition(":")
    if hasattr(engine, name):
        setattr(engine, name, on)
    else:
        getattr(ops, "set_" + name)(1 if on else int(off or 0))   # 1: the default routing


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--mc", type=int, default=100)
    ap.add_argument("--sonar", type=int, default=256)
    ap.add_argument("--only", type=int, choices=[0, 1], default=None,
                    help="run one setting (for a rocprofv3 kernel trace of it)")
    ap.add_argument("--train", action="store_true")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--flag", default="FOLD",
                    help="the engine switch the two arms set False / True (e.g. FOLD), or a "
                         "library routing switch ops.set_<flag> (e.g. expand16)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                    help="--train: trunk precision of the step")
    ap.add_argument("--tiles", type=int, nargs=2, default=None, metavar=("A", "B"),
                    help="--train: compare engine.FOLD_MIN_TILES A against B (fold on in both)")
    a = ap.parse_args()
    if a.train:
        return train_ab(a)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = define_models(None, 7, DEFAULT_PRIOR)["multimodal_model"].to(dev)
    x, b, s, _ = bench.synthetic_batch(a.batch, 224, a.sonar, dev, 99)
    hw = [(224, 224), (a.sonar, a.sonar), (a.sonar, a.sonar)]
    chunk = mc_chunk(model, a.batch, a.mc, dtype=torch.float16, device=dev, hw=hw)
    res = {False: [], True: []}
    outs = {}
    for r in range(a.rounds):
        order = (False, True) if r % 2 == 0 else (True, False)
        for fold in (order if a.only is None else (bool(a.only),)):
            _set(a.flag, fold)
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
    _set(a.flag, True)
    for f in (False, True):
        if not res[f]:
            continue
        t = min(res[f])
        print(f"fold={int(f)} best {a.mc * a.batch / t:.0f} MC-samples/s ({t * 1e3:.0f} ms), "
              f"mc_chunk {chunk}")
    if res[False] and res[True]:
        print(f"speedup {min(res[False]) / min(res[True]):.3f}x")


def train_ab(a):
    from mauv.engine import set_precision
    from mauv.optim import FusedAdam
    from mauv.train import mc_train_step
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = define_models(None, 7, DEFAULT_PRIOR)["multimodal_model"].to(dev)
    opt = FusedAdam(model.parameters(), lr=5e-5)
    crit = torch.nn.CrossEntropyLoss()
    B = 64
    x, b, s, y = bench.synthetic_batch(B, 224, a.sonar, dev, 1234)
    set_precision(model, torch.bfloat16 if a.dtype == "bf16" else None)
    kl_w = 2.0 ** 1 / 2.0 ** 30

    def step():
        return mc_train_step(model, (x, b, s), y, crit, opt, 5, B, kl_w)
    res = {False: [], True: []}
    for r in range(a.rounds):
        order = (False, True) if r % 2 == 0 else (True, False)
        for fold in (order if a.only is None else (bool(a.only),)):
            if a.tiles:   # arm False = FOLD_MIN_TILES A, arm True = B
                engine.FOLD, engine.FOLD_MIN_TILES = True, a.tiles[int(fold)]
            else:
                _set(a.flag, fold)
            for _ in range(2):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize()
            res[fold].append((time.perf_counter() - t0) / a.steps)
            print(f"round {r} fold={int(fold)}: {B / res[fold][-1]:.1f} triplets/s "
                  f"({res[fold][-1] * 1e3:.2f} ms/step)", flush=True)
    _set(a.flag, True)
    for f in (False, True):
        if res[f]:
            t = min(res[f])
            print(f"fold={int(f)} best {B / t:.1f} triplets/s ({t * 1e3:.2f} ms/step)")
    if res[False] and res[True]:
        print(f"speedup {min(res[False]) / min(res[True]):.3f}x")


if __name__ == "__main__":
    main()
