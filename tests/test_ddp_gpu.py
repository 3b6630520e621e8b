"""DistributedMC on the GPU engine: two ranks on one MI355X (gloo over CUDA tensors — RCCL
needs one GPU per rank, which the 8-GPU driver run provides).  The per-trunk all-reduces
issued from the engine's backward hook (overlapped with the other trunks' backward) give
bit-identical averaged gradients to the plain all-reduce after the backward, the ranks end
with identical gradients, and those are the mean of the ranks' local gradients."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "multimodal-auv_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from mauv.models import define_models, DEFAULT_PRIOR
    from mauv.ddp import DistributedMC
    from mauv.engine import root_state
    from mauv.kl import get_kl_loss
    from mauv import mchead
    from tests.golden.common import make_batches
    torch.manual_seed(0)
    model = define_models(None, 7, DEFAULT_PRIOR)["multimodal_model"].cuda()
    ddp = DistributedMC(model)
    st = root_state(model)
    b = make_batches(100 + rank, 1, B=2, S_opt=64, S_son=64)[0]
    x, ba, s, y = (b[k].cuda() for k in ("main_image", "bathy_image", "sss_image", "label"))

    def step(reduce):
        st.offset = 0
        for p in model.parameters():
            p.grad = None
        lg = ddp.mc_forward(x, ba, s, 2)
        ce, _, _ = mchead.mc_mean_ce(lg, y)
        (ce + get_kl_loss(ddp) / 2 * 0.5).backward()
        if reduce:
            ddp.allreduce_grads()
        torch.cuda.synchronize()
        return st.arena.flat.clone()

    hook = st.grad_ready_hook
    st.grad_ready_hook = None
    local = step(False)                      # this rank's own gradient
    plain = step(True)                       # all-reduced after the backward
    st.grad_ready_hook = hook
    overlapped = step(True)                  # trunk slices from the backward hook
    early = ddp.n_overlapped
    summed = local.clone()
    dist.all_reduce(summed)
    torch.save((torch.equal(overlapped, plain), (plain - summed / world).abs().max().item(),
                overlapped.sum().item(), overlapped.abs().sum().item(), early),
               os.path.join(q, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_overlapped_trunk_allreduce_on_gpu(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    res = [torch.load(os.path.join(tmp_path, f"r{r}.pt")) for r in range(2)]
    for same, err, _, _, early in res:
        assert same
        assert err <= 1e-6
        assert early >= 2   # at least two trunk slices went during the backward
    assert res[0][2] == res[1][2] and res[0][3] == res[1][3]
