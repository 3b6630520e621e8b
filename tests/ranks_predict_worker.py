"""Worker of tests/test_bench_ranks_gpu.py::test_mc_sharded_statistics_equal_single_rank (not a
test module): under torch.distributed.run (gloo; every rank on cuda:0) — or alone, world 1 —
build the tri-modal model from one seed, wrap it in DistributedMC when world > 1, and write
rank 0's MC statistics of one batch (num_mc over the ranks, f16 autocast first, then fp32) to
the JSON file named by argv[1]."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-auv_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main(out, num_mc=10, chunk=2):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group("gloo")
    rank = dist.get_rank() if world > 1 else 0
    torch.cuda.set_device(0)
    from mauv.models import define_models, DEFAULT_PRIOR
    from mauv.ddp import DistributedMC
    from mauv.engine import root_state
    from mauv.predict import mc_statistics, _shard_group
    from tests.golden.common import make_batches, SEED_DATA
    torch.manual_seed(0)
    m = define_models(None, 7, DEFAULT_PRIOR)["multimodal_model"].cuda()
    root_state(m).seed = 123456789
    w = DistributedMC(m) if world > 1 else m
    bt = make_batches(SEED_DATA + 3, 1, B=4, S_opt=64, S_son=64)[0]
    x, b, s = (bt[k].cuda() for k in ("main_image", "bathy_image", "sss_image"))
    res = {"world": world}
    for name, amp in (("f16", True), ("fp32", False)):
        with torch.no_grad(), torch.autocast("cuda", enabled=amp):
            st = mc_statistics(w, x, b, s, num_mc, chunk=chunk, group=_shard_group(w))
        res[name] = {k: st[k].double().cpu().tolist()
                     for k in ("pred", "var", "aleatoric", "predictive_entropy", "mean_prob")}
    if rank == 0:
        with open(out, "w") as fh:
            json.dump(res, fh)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
