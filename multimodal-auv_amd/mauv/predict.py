"""MC inference with the reference's call surface (inference/predictors.py:9-97).

``multimodal_predict_and_save`` writes the same CSV (``Image Name, Predicted Class,
Predictive Uncertainty, Aleatoric Uncertainty``) with the same maths (softmax per pass,
unbiased variance over the MC samples averaged over classes, aleatoric = mean entropy with
eps 1e-7, class = argmax of the mean probability) — but the ``num_mc_samples`` passes run as
batched launches (``mc_forward``, chunked to fit HBM) and the statistics are one fused
reduction (mauv_mc_stats / mauv_mc_finalize) whose partial sums all-reduce across ranks for
MC-sharded multi-GPU inference.

Numerics: like the reference (predictors.py:55) the MC passes run under
``torch.amp.autocast(device_type='cuda')``, which the engine follows with f16 trunks
(activations and sampled weights 16-bit, fp32 accumulation and BN statistics); the fusion head
and every reduction stay fp32/fp64.
"""
import collections
import csv
import logging
import math
import os

import torch
import torch.distributed as dist

from . import mchead
from .engine import root_state
from .kl import unwrap

# peak live activation channels per image of one MC sample, in units of the layer-1 grid
# (H/4 x W/4): a layer-1 bottleneck without saving holds its input (256), y1 and y2 (64 each),
# y3, the downsample residual and the output (256 each) -> 1152; the stem's conv output
# (64 ch at H/2 x W/2) is 256 of them.  The trunks run one after another in inference.
_PEAK_CH_L1 = 1152
_ALLOC_SLACK = 1.25   # caching-allocator rounding and the BN / statistics buffers


def mc_chunk(model, batch_size, num_mc, budget_bytes=None, hw=None, dtype=None, device=None):
    """How many MC samples to batch per launch for inference, from the activation footprint
    of the largest trunk input (``hw`` = [(H, W), ...] of the three images), the trunk storage
    dtype and the device memory actually available; chunks are balanced (100 samples at a
    limit of 22 -> five chunks of 20)."""
    core = unwrap(model)
    if budget_bytes is None:
        # 160 GiB / 60 % of the free HBM: the estimate below runs ~1.5x above the measured
        # peak (chunk 50 of the bench batch: 97 GiB), and larger chunks are faster (f16,
        # B=256, N=100: chunk 20 -> 10.8k, 34 -> 10.9k, 50 -> 11.0k MC-samples/s)
        budget_bytes = getattr(core, "mc_infer_budget_bytes", 160 << 30)
        dev = device if device is not None else _param_device(core)
        if dev is not None and dev.type == "cuda":
            free, _ = torch.cuda.mem_get_info(dev)
            cached = torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
            budget_bytes = min(budget_bytes, int(0.6 * (free + cached)))
    esize = torch.tensor([], dtype=dtype or torch.float32).element_size()
    hw = hw or [(256, 256)]
    grid = max(math.ceil(h / 4) * math.ceil(w / 4) for h, w in hw)
    per_sample = esize * _PEAK_CH_L1 * grid * batch_size * _ALLOC_SLACK
    limit = max(1, min(num_mc, int(budget_bytes // max(per_sample, 1))))
    n_chunks = math.ceil(num_mc / limit) if num_mc > 0 else 1
    return max(1, math.ceil(num_mc / n_chunks))


def _param_device(core):
    for p in core.parameters():
        return p.device
    return None


# Small MC chunks (the reference's own call shape: batch_size_unimodal=8, num_mc=12,
# main.py:261-271,310,315) are launch-bound: ~1,000 C-ABI launches per tri-modal forward from
# Python.  Their forward is captured once per shape into a HIP graph and replayed; the MC
# samples stay fresh on every replay because the sampling kernels read their sample index from
# a device counter (mauv_reparam_sample_ex).  MAUV_GRAPH_INFER=0 turns it off; chunks above
# the activation budget below always run eagerly (a graph's pool keeps its activations).
GRAPH_INFER = os.environ.get("MAUV_GRAPH_INFER", "1") == "1"
_GRAPH_MAX_BYTES = 6 << 30


class _GraphedChunk:
    """One captured MC-chunk forward: static inputs in, static [G, B, C] logits out."""

    def __init__(self, core, inputs, G):
        st = root_state(core)
        dev = inputs[0].device
        self.core, self.G = core, G
        self.static = [t.clone() for t in inputs]
        self.base = torch.zeros(1, dtype=torch.int64, device=dev)
        self.graph = torch.cuda.CUDAGraph()
        saved = st.offset
        st.sample_base, st.offset = self.base, 0      # captured with sample0 = 0 + *base
        try:
            with torch.cuda.graph(self.graph):
                self.out = core.mc_forward(*self.static, G)
        finally:
            st.sample_base, st.offset = None, saved

    def __call__(self, inputs):
        st = root_state(self.core)
        for d, x in zip(self.static, inputs):
            d.copy_(x)
        self.base.fill_(st.next_samples(self.G))       # this chunk's MC sample indices
        self.graph.replay()
        return self.out


_GRAPH_CACHE_MAX = 2   # captured chunk graphs kept per model (each holds a private pool)


def _graph_state_key(base, st):
    """What a capture bakes in besides the input shapes: the Philox seed (a kernel scalar), the
    BN mode / momentum / eps of every BatchNorm (batch statistics + running-stat updates vs
    eval parameters) and the storage of every parameter and buffer (a ``p.data = ...`` rebind,
    bayesian-torch's MOPED idiom, leaves a replay reading freed memory)."""
    bns = st.plist("graph_bns", lambda: [m for m in base.modules()
                                         if isinstance(m, torch.nn.modules.batchnorm._BatchNorm)])
    tensors = st.plist("graph_tensors", lambda: list(base.parameters()) + list(base.buffers()))
    return (st.seed, base.training, tuple((m.training, m.momentum, m.eps) for m in bns),
            hash(tuple(t.data_ptr() for t in tensors)))


def drop_graphs(model):
    """Release the captured inference graphs of ``model`` (and their memory pools)."""
    base = unwrap(model)
    base.__dict__.pop("_mauv_graphs", None)
    base.__dict__.pop("_mauv_graph_seen", None)


def _chunk_forward(core, inputs, G):
    """core.mc_forward(*inputs, G), through a captured HIP graph for small chunks once a shape
    has run eagerly (the first run also loads every kernel the capture records).  The cache is
    keyed on the shapes and on everything the capture fixes (``_graph_state_key``) and keeps the
    ``_GRAPH_CACHE_MAX`` most recently used graphs."""
    if not GRAPH_INFER or torch.is_grad_enabled() or not inputs[0].is_cuda:
        return core.mc_forward(*inputs, G)
    base = unwrap(core)
    st = root_state(base)
    if st.eps_provider is not None:                    # tests feed explicit epsilons: eager
        return base.mc_forward(*inputs, G)
    dt = st.trunk_dtype()
    B = inputs[0].shape[0]
    per = mc_chunk_bytes(B, dt, [t.shape[-2:] for t in inputs])
    if per * G > _GRAPH_MAX_BYTES:
        return base.mc_forward(*inputs, G)
    key = (tuple(tuple(t.shape) for t in inputs), tuple(t.dtype for t in inputs), G, dt,
           inputs[0].device, _graph_state_key(base, st))
    cache = base.__dict__.setdefault("_mauv_graphs", collections.OrderedDict())
    g = cache.get(key)
    if g is None:
        seen = base.__dict__.setdefault("_mauv_graph_seen", set())
        if key not in seen:
            seen.add(key)
            return base.mc_forward(*inputs, G)
        while len(cache) >= _GRAPH_CACHE_MAX:
            cache.popitem(last=False)
        g = cache[key] = _GraphedChunk(base, inputs, G)
    cache.move_to_end(key)
    return g(inputs)


def mc_chunk_bytes(batch_size, dtype, hw):
    """Estimated peak activation bytes of one MC sample of one inference forward."""
    esize = torch.tensor([], dtype=dtype or torch.float32).element_size()
    grid = max(math.ceil(h / 4) * math.ceil(w / 4) for h, w in hw)
    return esize * _PEAK_CH_L1 * grid * batch_size * _ALLOC_SLACK


def local_mc_count(num_mc, rank, world):
    """MC samples this rank draws when ``num_mc`` are sharded over ``world`` ranks."""
    return num_mc // world + (1 if rank < num_mc % world else 0)


def mc_statistics(model, inputs, bathy, sss, num_mc, eps_h=1e-7, eps_pred=1e-8, chunk=None,
                  group=None):
    """Fused MC statistics for one batch; with ``group`` (torch.distributed), the MC samples
    are sharded across ranks (each rank: full batch, ~num_mc/world samples; BN statistics
    stay per-sample exactly as in the reference) and the sums all-reduced once.  Sharded, rank
    r draws MC samples [s0 + sum of the lower ranks' counts, + its own count) of the rank-0
    Philox stream (``shared_seed``, DistributedMC), s0 = the sample counter at the call (equal
    on every rank of a rank-symmetric program): the union is exactly the single-rank draw, so
    the statistics do not depend on the world size (up to the float64 sum order)."""
    B = inputs.shape[0]
    rank, world = (dist.get_rank(group), dist.get_world_size(group)) if group is not None \
        else (0, 1)
    local = local_mc_count(num_mc, rank, world)
    core = model if hasattr(model, "mc_forward") else unwrap(model)
    st = root_state(unwrap(model))
    shard = group is not None and world > 1 and getattr(st, "shared_seed", None) is not None
    if shard:
        s0, seed = st.offset, st.seed
        st.seed = st.shared_seed
        st.offset = s0 + sum(local_mc_count(num_mc, q, world) for q in range(rank))
        try:
            return _mc_statistics_local(model, core, inputs, bathy, sss, num_mc, local, eps_h,
                                        eps_pred, chunk, group)
        finally:
            st.seed, st.offset = seed, s0 + num_mc
    return _mc_statistics_local(model, core, inputs, bathy, sss, num_mc, local, eps_h, eps_pred,
                                chunk, group)


def _mc_statistics_local(model, core, inputs, bathy, sss, num_mc, local, eps_h, eps_pred, chunk,
                         group):
    B = inputs.shape[0]
    if chunk is None:
        dt = root_state(unwrap(model)).trunk_dtype()
        chunk = mc_chunk(model, B, max(local, 1), dtype=dt, device=inputs.device,
                         hw=[t.shape[-2:] for t in (inputs, bathy, sss)])
    sums = None
    done = 0
    while done < local:
        g = min(chunk, local - done)
        logits = _chunk_forward(core, (inputs, bathy, sss), g)
        sums = mchead.mc_stats(logits, eps_h, sums)
        done += g
        del logits
    C = unwrap(model).fc2.out_features
    if sums is None:
        sums = torch.zeros(B, 2 * C + 1, dtype=torch.float64, device=inputs.device)
    if group is not None:
        dist.all_reduce(sums, group=group)
    return mchead.mc_finalize(sums, num_mc, C, eps_pred)


def _shard_group(model):
    """MC samples shard across ranks when the model is wrapped in mauv.ddp.DistributedMC (each
    rank then passes the same batches); a bare model predicts alone."""
    if getattr(model, "_mauv_wrapper", False) and dist.is_available() and dist.is_initialized() \
            and getattr(model, "world", 1) > 1:
        return model.group if model.group is not None else dist.group.WORLD
    return None


def multimodal_predict_and_save(multimodal_model, dataloader, device, csv_path,
                                num_mc_samples=10, sss_patch_type="", channel_patch_type="",
                                model_type="multimodal"):
    """inference/predictors.py:9-97 (model kept in .train(): BN uses batch statistics; MC
    passes under torch.amp.autocast as predictors.py:55 -> f16 trunks on a ROCm device)."""
    from .train import loop_device, is_writer, _NullFile, _tile_to
    device = torch.device(loop_device(multimodal_model, device))
    amp_device = "cuda" if device.type == "cuda" else "cpu"
    group = _shard_group(multimodal_model)
    writer = is_writer(multimodal_model)   # MC-sharded: every rank holds the same rows
    multimodal_model.train()
    logging.info(f"CSV will be saved to: {csv_path}")
    with (open(csv_path, mode="w", newline="") if writer else _NullFile()) as fh:
        w = csv.writer(fh)
        w.writerow(["Image Name", "Predicted Class", "Predictive Uncertainty",
                    "Aleatoric Uncertainty"])
        with torch.no_grad():
            for batch_idx, (inputs, bathy, sss, image_name) in enumerate(dataloader):
                inputs = _tile_to(inputs, device, optical=True)   # uint8 tiles: staged
                bathy = _tile_to(bathy, device)                    # on the device
                sss = _tile_to(sss, device)
                if hasattr(unwrap(multimodal_model), "mc_forward"):
                    if group is not None:
                        multimodal_model.check_same_batch(inputs.size(0))
                    with torch.amp.autocast(device_type=amp_device):
                        st = mc_statistics(multimodal_model, inputs, bathy, sss,
                                           num_mc_samples, group=group)
                    pred, var, alea = st["pred"], st["var"], st["aleatoric"]
                else:  # foreign model: reference sequential loop
                    probs = []
                    for _ in range(num_mc_samples):
                        with torch.amp.autocast(device_type=amp_device):
                            probs.append(torch.softmax(multimodal_model(inputs, bathy, sss), 1))
                    P = torch.stack(probs).float()
                    var = torch.var(P, dim=0).mean(dim=1)
                    alea = torch.mean(-torch.sum(P * torch.log(P + 1e-7), dim=-1), dim=0)
                    pred = torch.argmax(P.mean(0), dim=1)
                pred, var, alea = pred.cpu().tolist(), var.cpu().tolist(), alea.cpu().tolist()
                for i in range(inputs.size(0)):
                    name = image_name[i] if isinstance(image_name, (list, tuple)) else image_name
                    w.writerow([name, pred[i], var[i], alea[i]])
    logging.info("Completed: multimodal_predict_and_save")
