"""Data-parallel training over RCCL (one process per GPU), replacing the reference's
single-process ``nn.DataParallel`` (utils/device.py:19).

The reference replicates every parameter and buffer to every GPU inside every forward call
(DataParallel.replicate), scatters the batch, gathers logits to GPU 0 and reduce-adds the
gradients in backward.  Here each rank owns a full model, runs its own minibatch shard with
its own Philox epsilon stream (as each DataParallel replica samples its own epsilons) and its
own BN batch statistics (as each replica normalises its own chunk), and gradients meet in
bucketed all-reduces of the flat gradient arena (146.8 M fp32 = 587 MB per step) over xGMI.
Parameters are broadcast from rank 0 once at wrap time.

Overlap: the three ResNet-50 trunks run their backward on streams of their own and own
contiguous slices of the arena (~47 M floats each).  When a trunk's backward has written its
last gradient, the engine calls ``grad_ready_hook`` on that trunk's stream and its slice
all-reduces (async, 64 MB buckets) while the other trunks are still in backward; the fusion
head's slice and any trunk that finished before the KL backward (which writes every slice)
go in ``allreduce_grads`` after the backward.  The order of collectives is the autograd
order of the trunk nodes, identical on every rank.

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

    def __init__(self, module, group=None, bucket_bytes=64 << 20, overlap=True,
                 grad_dtype=torch.float32):
        """grad_dtype=torch.bfloat16: the gradient exchange moves a bf16 copy of the arena
        (146.8 M values = 294 MB per step instead of 587 MB, SURVEY §8e's bf16 figure): each
        slice is rounded to bf16, all-reduced, widened back into the fp32 arena and averaged
        there; the optimiser's master gradients stay fp32."""
        super().__init__()
        self.module = module
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        assert grad_dtype in (torch.float32, torch.bfloat16)
        self.grad_dtype = grad_dtype
        self.bucket_elems = max(1, bucket_bytes // (4 if grad_dtype == torch.float32 else 2))
        self._lp = None          # bf16 exchange buffer (grad_dtype bf16)
        self._lp_ranges = []     # [start, end) slices whose bf16 sums await widening
        self.overlap = overlap
        with torch.no_grad():
            for t in list(module.parameters()) + list(module.buffers()):
                dist.broadcast(t.data, src=dist.get_global_rank(group, 0) if group else 0,
                               group=group)
        st = root_state(module)
        # training: each rank its own Philox stream (as each DataParallel replica samples its
        # own epsilons); MC-sharded inference draws from the rank-0 stream instead
        # (predict.mc_statistics), so a sharded prediction equals the single-rank one
        st.shared_seed = st.seed
        st.seed = (st.seed + 0x9E3779B97F4A7C15 * (self.rank + 1)) % (1 << 62)
        self._pending = []      # async works of the trunk slices issued during backward
        self._done = []         # [start, end) arena ranges they cover
        self._kl_mark = 0
        self.n_overlapped = 0   # trunk slices all-reduced from the backward hook (cumulative)
        self.n_buckets = 0      # all-reduce calls of the gradient exchange (cumulative)
        self.elems_reduced = 0  # arena values exchanged (cumulative)
        if overlap and self.world > 1:
            st.grad_ready_hook = self._trunk_ready

    # ---- forward: the model's, unchanged ----
    def forward(self, *args, **kw):
        self._begin_step()
        return self.module(*args, **kw)

    def mc_forward(self, *args, **kw):
        self._begin_step()
        return self.module.mc_forward(*args, **kw)

    def _begin_step(self):
        if torch.is_grad_enabled():
            self._kl_mark = root_state(self.module).kl_bwd_count

    # ---- gradient exchange ----
    def _slice_of(self, trunk):
        """[start, end) of ``trunk``'s parameters in the flat arena (contiguous by the
        parameter order of the model), or None."""
        st = root_state(self.module)
        arena = st.arena
        ids = {id(p) for p in trunk.parameters() if p.requires_grad}
        idx = [i for i, p in enumerate(arena.params) if id(p) in ids]
        if not idx or idx != list(range(idx[0], idx[-1] + 1)):
            return None
        start = arena.offsets[idx[0]]
        end = arena.offsets[idx[-1] + 1] if idx[-1] + 1 < len(arena.offsets) else arena.numel
        return start, end

    def _allreduce_range(self, flat, start, end, async_op):
        buf = flat
        if self.grad_dtype == torch.bfloat16:
            if self._lp is None or self._lp.numel() != flat.numel() or \
                    self._lp.device != flat.device:
                self._lp = torch.empty(flat.numel(), dtype=torch.bfloat16, device=flat.device)
            buf = self._lp
            buf[start:end].copy_(flat[start:end])     # round to bf16 on the current stream
            self._lp_ranges.append((start, end))
        works = []
        self.elems_reduced += end - start
        for off in range(start, end, self.bucket_elems):
            self.n_buckets += 1
            w = dist.all_reduce(buf[off:min(end, off + self.bucket_elems)], group=self.group,
                                async_op=async_op)
            if async_op:
                works.append(w)
        return works

    def _widen(self, flat):
        """bf16 exchange: the summed slices back into the fp32 arena (exact widening)."""
        for a, b in self._lp_ranges:
            flat[a:b].copy_(self._lp[a:b])
        self._lp_ranges = []

    def _trunk_ready(self, trunk):
        """Engine hook (trunk stream current): all-reduce this trunk's arena slice now, unless
        the KL backward — which adds into every slice — has not been issued yet this step."""
        st = root_state(self.module)
        if st.kl_bwd_count <= self._kl_mark:   # the loops always add get_kl_loss (:114)
            return
        rng = self._slice_of(trunk)
        if rng is None:
            return
        # the KL backward was issued on the caller's stream and adds into this slice: order
        # the all-reduce after it explicitly (not by autograd's node order)
        if st.kl_bwd_event is not None:
            torch.cuda.current_stream().wait_event(st.kl_bwd_event)
        self._pending += self._allreduce_range(st.arena.flat, *rng, async_op=True)
        self._done.append(rng)
        self.n_overlapped += 1

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

    def all_ranks_device(self, flag):
        """In-place MIN of a device int32 flag over the group, stream-ordered (no host sync):
        the device-gated training step (mauv.train.mc_train_step) skips on every rank or none."""
        if self.world > 1:
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)

    def sum_ranks(self, values):
        """Element-wise sum of a list of floats over the ranks (one float64 all-reduce)."""
        if self.world == 1:
            return list(values)
        dev = next(self.module.parameters()).device
        t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=dev)
        dist.all_reduce(t, group=self.group)
        return t.cpu().tolist()

    def check_same_batch(self, B):
        """MC-sharded prediction all-reduces per-item statistics: every rank must hold the same
        batch.  One MAX all-reduce of (B, -B) checks that the batch sizes agree."""
        if self.world == 1:
            return
        dev = next(self.module.parameters()).device
        t = torch.tensor([B, -B], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        lo, hi = -int(t[1]), int(t[0])
        if lo != hi:
            raise RuntimeError(f"mauv MC-sharded prediction: ranks hold batches of different "
                               f"sizes ({lo}..{hi}); every rank must iterate the same loader in "
                               "the same order (the MC samples, not the images, are sharded)")

    def allreduce_grads(self):
        """Average the flat gradient arena across ranks: wait for the trunk slices issued
        during backward, all-reduce the rest in buckets, scale by 1/world."""
        st = root_state(self.module)
        if self.world == 1:
            self._pending, self._done = [], []
            return
        if st.arena is None:   # a foreign module (no engine arena): reduce its p.grad tensors
            for p in self.module.parameters():
                if p.grad is not None:
                    dist.all_reduce(p.grad, group=self.group)
                    p.grad.mul_(1.0 / self.world)
            return
        flat = st.arena.flat
        for w in self._pending:
            w.wait()
        done = sorted(self._done)
        self._pending, self._done = [], []
        cur = 0
        for a, b in done + [(flat.numel(), flat.numel())]:
            if cur < a:
                self._allreduce_range(flat, cur, a, async_op=False)
            cur = max(cur, b)
        if self.grad_dtype == torch.bfloat16:
            self._widen(flat)
        flat.mul_(1.0 / self.world)

    def state_dict(self, *a, **k):
        return self.module.state_dict(*a, **k)

    def load_state_dict(self, *a, **k):
        return self.module.load_state_dict(*a, **k)
