"""Data-parallel training over RCCL (one process per GPU), replacing the reference's
single-process ``nn.DataParallel`` (utils/device.py:19).

The reference replicates every parameter and buffer to every GPU inside every forward call
(DataParallel.replicate), scatters the batch, gathers logits to GPU 0 and reduce-adds the
gradients in backward.  Here each rank owns a full model, runs its own minibatch shard with
its own Philox epsilon stream (as each DataParallel replica samples its own epsilons) and its
own BN batch statistics (as each replica normalises its own chunk), and gradients meet in
ONE bucketed all-reduce of the flat gradient arena per step (146.8 M fp32 = 587 MB) over
xGMI.  Parameters are broadcast from rank 0 once at wrap time.

``DistributedMC`` deliberately does not subclass DistributedDataParallel: the reference's
loops special-case DDP by calling ``model.module(...)`` (train/multimodal.py:109-110), which
would skip gradient synchronisation; with this wrapper they take the ordinary branch.
"""
import torch
import torch.distributed as dist
import torch.nn as nn

from .engine import root_state


class DistributedMC(nn.Module):
    _mauv_wrapper = True

    def __init__(self, module, group=None, bucket_bytes=64 << 20):
        super().__init__()
        self.module = module
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.bucket_elems = max(1, bucket_bytes // 4)
        with torch.no_grad():
            for t in list(module.parameters()) + list(module.buffers()):
                dist.broadcast(t.data, src=dist.get_global_rank(group, 0) if group else 0,
                               group=group)
        st = root_state(module)
        st.seed = (st.seed + 0x9E3779B97F4A7C15 * (self.rank + 1)) % (1 << 62)

    def forward(self, *args, **kw):
        return self.module(*args, **kw)

    def mc_forward(self, *args, **kw):
        return self.module.mc_forward(*args, **kw)

    def all_ranks(self, flag):
        """Logical AND of a per-rank decision over the group (one tiny all-reduce): the
        training loop skips a batch on every rank or on none, so the gradient all-reduces of
        later steps stay paired (the reference's DataParallel has one global loss)."""
        if self.world == 1:
            return bool(flag)
        dev = next(self.module.parameters()).device
        t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return bool(t.item())

    def allreduce_grads(self):
        """Average the flat gradient arena across ranks (bucketed RCCL all-reduce)."""
        st = root_state(self.module)
        if st.arena is None or self.world == 1:
            return
        flat = st.arena.flat
        n = flat.numel()
        for off in range(0, n, self.bucket_elems):
            dist.all_reduce(flat[off:off + self.bucket_elems], group=self.group)
        flat.mul_(1.0 / self.world)

    def state_dict(self, *a, **k):
        return self.module.state_dict(*a, **k)

    def load_state_dict(self, *a, **k):
        return self.module.load_state_dict(*a, **k)
