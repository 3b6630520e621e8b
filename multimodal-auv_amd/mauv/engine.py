"""MC-batched execution engine: compiles the tri-modal Bayesian model into HIP launches.

What the reference does (train/multimodal.py:107-118, inference/predictors.py:54-65):
``for _ in range(num_mc): model(inputs, bathy, sss)`` — N sequential stochastic forwards, each
re-sampling every Bayesian weight (bayesian-torch ``eps.normal_()``) and each running
BatchNorm in training mode on its own batch statistics, then one ``loss.backward()`` through
the N graphs.

What this engine does: one pass over the network in which every layer is ONE launch for all
N samples (G = N groups on blockIdx.z of the implicit-GEMM kernels), with per-group weights
``W_g = mu + softplus(rho) * eps_g`` (eps_g regenerated from Philox in the backward instead of
stored), per-group BN statistics and sequential running-stat updates, and a hand-scheduled
backward that writes dmu/drho/dgamma/dbeta straight into a flat gradient arena (one buffer
per model, so the data-parallel all-reduce is a single bucketed RCCL call).

Activations are NHWC ``[G][B][H][W][C]`` fp32.  The stems read one NHWC copy of the caller's
NCHW images with the channels zero-padded to 4 (16-bit path: 8), shared by all MC samples
(group stride 0).
"""
import os

import torch

from . import ops
from .layers import is_bayesian, LinearReparameterization


# The three trunks of MultiModalModel are independent until the fusion head: each runs its
# forward and (autograd replays the forward's stream) its backward on a stream of its own, so
# one trunk's memory-bound BN passes overlap another's MFMA-bound convs (MAUV_TRUNK_STREAMS=0:
# one stream, for serial kernel traces).
TRUNK_STREAMS = os.environ.get("MAUV_TRUNK_STREAMS", "1") == "1"
# Measured-positive schedule choices whose predecessors were removed (DESIGN.md §2.3, §2.8,
# §2.13): the stems run as ONE GEMM over im2col rows shared by the G samples (stem.hip) and their
# bn1 + ReLU is applied inside the max-pool's loads; training block outputs (bn3 + residual +
# ReLU) write 1-bit ReLU masks that their backward reads instead of the stored output; a block
# output's residual gradient dres = dout * mask is never written (the conv1 data gradient adds
# dout under the mask bits, the downsample BN's backward reads dout with them).  RES_MASK is not
# a switch: tests set it False to compare with the path that stores dres (bit-identical).
RES_MASK = True
# A 16-bit block output is not a separate pass: the next block's conv1 forms relu(bn3(y3) +
# residual) while loading its tiles and writes it through once, with its ReLU-mask bits when a
# backward will read them (ops.conv2d_fwd_fold) — where the launch has at least
# FOLD_MIN_TILES 256-row tiles (two rounds of the chip's CUs; fewer ran slower than the two
# passes).  Test hooks like RES_MASK: tests set FOLD False to compare with bn_apply + conv1
# (bit-identical) and FOLD_MIN_TILES 0 to fold their small shapes.
FOLD = True
FOLD_MIN_TILES = 512
# fp32 training: the BatchNorm-backward partial sums (sum dz, sum dz * xhat per channel) of a BN
# whose output gradient a data gradient produces are summed in that data gradient's LDS-staged
# epilogue (conv_common.h staged_epilogue_f32 + BP), so the partial pass over (y, dout) is not
# run: bn2 / bn1 from the conv3 / conv2 data gradients, the previous block's bn3 from conv1's
# (whose epilogue already adds the residual gradient; not where a downsample branch accumulates
# into that dx afterwards).  Test hook like FOLD: the same sums in another fp32 order.
BWD_PARTIALS_F32 = True
# 16-bit trunks: a conv output consumed by a batch-statistics BatchNorm is stored centred,
# y - c (ops.conv2d_fwd ysh: the accumulators start at -c, so the statistics partials are those
# of the stored values; the finalize updates the running mean with the true one), c = that BN's running mean as of the model's
# last refresh_centres (the model's first 16-bit forward, and the start of every training epoch
# of the drop-in loops) where it dominates the channel's spread.  The f16 / bf16 rounding error
# of the stored tensor then follows the batch spread |y - mean| instead of |y|: the largest of
# the path's rounding points.  Exact in real arithmetic; c changes only when
# refreshed, so predictions stay a function of the weights, samples and inputs (two predictor
# calls on the same samples give the same rows).  Test hook like FOLD.
CENTRE_Y = os.environ.get("MAUV_CENTRE_Y", "1") == "1"
# a channel is centred where |running mean| > this many running standard deviations
CENTRE_MIN_Z = float(os.environ.get("MAUV_CENTRE_MIN_Z", "1"))
_STREAMS = {}


def _first(v):
    """A conv attribute as one int (bayesian-torch keeps kernel_size an int, torch a tuple)."""
    return v if isinstance(v, int) else v[0]


def _trunk_streams(dev):
    """The streams of the three trunks."""
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _STREAMS:
        _STREAMS[key] = [torch.cuda.Stream(device=dev) for _ in range(3)]
    return _STREAMS[key]


# ----------------------------------------------------------------------------- root state
class GradArena:
    """Flat fp32 gradient buffer; every ``p.grad`` is a view into it.  Each view starts on a
    16-byte boundary (offsets rounded up to 4 floats; the gaps stay zero), as the fused Adam's
    and the NaN scan's 16-byte vector loads require."""

    ALIGN = 4

    def __init__(self, params, device):
        self.params = [p for p in params if p.requires_grad]
        offs, off = [], 0
        for p in self.params:
            offs.append(off)
            off += (p.numel() + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.numel = off
        self.flat = torch.zeros(self.numel, device=device)
        self.views = [self.flat[o:o + p.numel()].view_as(p) for p, o in zip(self.params, offs)]
        self.offsets = offs

    def ensure(self):
        ptrs_none = [p.grad is None for p in self.params]
        if all(ptrs_none):
            self.flat.zero_()
            for p, v in zip(self.params, self.views):
                p.grad = v
            return
        for p, v, none in zip(self.params, self.views, ptrs_none):
            if none:
                v.zero_()
                p.grad = v
            elif p.grad.data_ptr() != v.data_ptr():
                v.copy_(p.grad)
                p.grad = v


class RootState:
    """Per-model engine state: Philox layer ids, the MC sample counter, the grad arena."""

    def __init__(self, root):
        self.ids = {}
        for m in root.modules():
            if is_bayesian(m):
                self.ids[id(m)] = len(self.ids)
        self.params = list(root.parameters())
        self.seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self.offset = 0
        self.arena = None
        self.eps_provider = None  # tests: fn(module, name, G) -> [G, numel] tensor or None
        self.anchor = torch.zeros((), requires_grad=True)
        # "reference": bayesian-torch 0.5.0 rho-gradient (every MC pass sees the epsilon of
        # the LAST forward before backward — its eps buffer is overwritten in place while
        # autograd still references it); "exact": per-sample reparameterisation gradient.
        self.rho_grad = "reference"
        # trunk activation/weight storage: None = follow torch.autocast (the reference's
        # predictor runs under torch.amp.autocast, inference/predictors.py:55), else a dtype
        self.precision = None
        # data-parallel hooks (mauv.ddp.DistributedMC): called with a trunk module when that
        # trunk's backward has written its last gradient (on the trunk's stream), so its
        # slice of the arena can be all-reduced while the other trunks still run backward;
        # kl_bwd_count counts issued KL backwards (they write into every trunk's slice)
        self.grad_ready_hook = None
        self.kl_bwd_count = 0
        self.kl_bwd_event = None   # recorded after the last KL backward (mauv.kl)
        # device int64 [1] added to every sampled MC index while a forward is being captured
        # into a HIP graph (mauv.predict): the replay draws fresh samples after it is updated
        self.sample_base = None
        # parameter lists the entry points walk every call (named_parameters over 696 tensors:
        # ~1.3 ms of host time per step ahead of the first kernel); built once, like self.params
        self._plists = {}
        # centred 16-bit storage (CENTRE_Y): the BatchNorms that track running statistics and one
        # flat buffer of their running means as of the last refresh_centres (views per BN)
        self.bns = [m for m in root.modules()
                    if isinstance(m, torch.nn.modules.batchnorm._BatchNorm)
                    and m.track_running_stats and m.running_mean is not None]
        self._centre_buf = None
        self._centre_views = {}

    def refresh_centres(self):
        """Every tracked BatchNorm's centre from its running statistics: the running mean where
        it exceeds CENTRE_MIN_Z running standard deviations, else 0 — centring pays where a
        channel's mean dominates its spread (the stored magnitude |y| ~ |mean| + std falls to
        ~std) and only adds the running mean's staleness elsewhere."""
        if not self.bns:
            return
        dev = self.bns[0].running_mean.device
        if self._centre_buf is None or self._centre_buf.device != dev:
            n = sum(bn.running_mean.numel() for bn in self.bns)
            self._centre_buf = torch.empty(n, device=dev)
            off, views = 0, {}
            for bn in self.bns:
                c = bn.running_mean.numel()
                views[id(bn)] = self._centre_buf[off:off + c]
                off += c
            self._centre_views = views
        with torch.no_grad():
            rm = torch.cat([bn.running_mean.detach().float() for bn in self.bns])
            rv = torch.cat([bn.running_var.detach().float() if bn.running_var is not None
                            else torch.zeros_like(bn.running_mean) for bn in self.bns])
            keep = rm.abs() > CENTRE_MIN_Z * rv.clamp(min=0).sqrt()
            torch.where(keep, rm, torch.zeros_like(rm), out=self._centre_buf)

    def centre(self, bn):
        """bn's centre (the first call builds the buffer from the current running means)."""
        if self._centre_buf is None or self._centre_buf.device != bn.running_mean.device:
            self.refresh_centres()
        return self._centre_views.get(id(bn))

    def plist(self, key, build):
        got = self._plists.get(key)
        if got is None:
            got = self._plists[key] = build()
        return got

    def trunk_dtype(self):
        if self.precision is not None:
            return self.precision
        if torch.is_autocast_enabled("cuda"):
            dt = torch.get_autocast_dtype("cuda")
            if dt in (torch.bfloat16, torch.float16):
                return dt
        return torch.float32

    def layer_id(self, m, bias=False):
        return 2 * self.ids[id(m)] + int(bias)

    def next_samples(self, G):
        s = self.offset
        self.offset += G
        return s

    def grads(self, device):
        if self.arena is None or self.arena.flat.device != device:
            self.arena = GradArena(self.params, device)
        self.arena.ensure()
        return self.arena


def root_state(root):
    st = root.__dict__.get("_mauv_state")
    if st is None:
        st = RootState(root)
        root.__dict__["_mauv_state"] = st
    return st


def invalidate(root):
    root.__dict__.pop("_mauv_state", None)


def refresh_centres(root):
    """Take the 16-bit trunks' storage centres (CENTRE_Y) from the current BatchNorm running
    statistics — the drop-in training loops do at every epoch; the first 16-bit forward of a
    model takes them on its own."""
    root_state(root).refresh_centres()


def set_rho_grad_mode(root, mode):
    """"reference" (default; bayesian-torch 0.5.0 behaviour) or "exact"."""
    assert mode in ("reference", "exact")
    root_state(root).rho_grad = mode


def set_precision(root, dtype):
    """Storage/compute format of the three trunks: torch.float32 (exact fp32 MFMA),
    torch.bfloat16 (BASELINE configs[2] training) or torch.float16 (16-bit MFMA, fp32
    accumulation, BN statistics, weight gradients and master parameters); None follows
    torch.autocast("cuda") like the reference's own ops do.  The fusion head is fp32."""
    assert dtype in (None, torch.float32, torch.bfloat16, torch.float16)
    root_state(root).precision = dtype


def needs_grad(params):
    return torch.is_grad_enabled() and any(p.requires_grad for p in params)


class _Engine(torch.autograd.Function):
    """Autograd node around a runner: forward = the HIP schedule; backward = the reverse
    HIP schedule, which writes parameter gradients into the arena directly."""

    @staticmethod
    def forward(ctx, runner, anchor, *inputs):
        ctx.runner = runner
        return runner.run_forward(*inputs)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, *grads):
        runner, ctx.runner = ctx.runner, None
        gins = runner.run_backward(*grads)
        return (None, None) + tuple(gins)


# ----------------------------------------------------------------------------- base runner
class _Runner:
    def __init__(self, state, G, sample0, save):
        self.st, self.G, self.s0, self.save = state, G, sample0, save

    def _eps(self, m, name):
        """Explicit epsilons from a test provider (None: Philox).  Asked once per layer and
        runner: the backward reuses the forward's draw, as Philox regenerates the same one."""
        fn = self.st.eps_provider
        if fn is None:
            return None
        cache = self.__dict__.setdefault("_eps_cache", {})
        key = (id(m), name)
        if key not in cache:
            cache[key] = fn(m, name, self.G)
            # the layer's latest draw, for a reference-mode rho-gradient of an EARLIER forward
            # (sequential grad-enabled calls before one backward, the noise Examples' loop)
            self.st.__dict__.setdefault("eps_last", {})[key] = (self.s0, cache[key])
        return cache[key]

    # ---- Bayesian parameter sampling (mauv_reparam_sample) ----
    def _sample(self, m, mu, rho, name, out, Cout, Cin, RS, bias=False, out_gstride=0,
                cin_pad=None):
        if self.st.sample_base is not None:   # inside a captured inference graph (predict.py)
            ops.reparam_sample_ex(mu, rho, out, self.G, self.st.seed, self.s0,
                                  self.st.sample_base, self.st.layer_id(m, bias), Cout, Cin, RS,
                                  eps=self._eps(m, name), out_gstride=out_gstride,
                                  cin_pad=cin_pad)
            return
        ops.reparam_sample(mu, rho, out, self.G, self.st.seed, self.s0,
                           self.st.layer_id(m, bias), Cout, Cin, RS, eps=self._eps(m, name),
                           out_gstride=out_gstride, cin_pad=cin_pad)

    def _reparam_bwd(self, m, mu, rho, dw, splits, Cout, Cin, RS, name, bias=False,
                     dw_gstride=0, dw_sstride=0, dw_cin=None):
        if not mu.requires_grad:
            return
        fixed = self.st.offset - 1 if self.st.rho_grad == "reference" else -1
        eps, s0 = self._eps(m, name), self.s0
        if eps is not None and fixed >= 0 and not s0 <= fixed < s0 + self.G:
            # explicit epsilons whose last draw belongs to a later forward: its rows
            ls0, leps = self.st.eps_last[(id(m), name)]
            if not ls0 <= fixed < ls0 + leps.shape[0]:
                raise RuntimeError(
                    f"mauv: the reference-mode rho gradient of {name} needs the epsilon of MC "
                    f"sample {fixed}, but this layer's last explicit draw covers samples "
                    f"{ls0}..{ls0 + leps.shape[0] - 1} (a forward skipped this layer)")
            eps, s0 = leps[fixed - ls0:fixed - ls0 + 1], fixed
        ops.reparam_bwd(dw, splits, mu, rho, mu.grad, rho.grad, self.G, self.st.seed, s0,
                        self.st.layer_id(m, bias), Cout, Cin, RS, eps=eps,
                        dw_gstride=dw_gstride, dw_sstride=dw_sstride, fixed_sample=fixed,
                        dw_cin=dw_cin)

    # ---- linear = 1x1 conv on [G][rows][K] ----
    def _linear(self, lin, x, rows):
        G, N, K = self.G, lin.out_features, lin.in_features
        w = torch.empty(G, N, K, device=x.device)
        self._sample(lin, lin.mu_weight, lin.rho_weight, "weight", w, N, K, 1)
        b = None
        if lin.mu_bias is not None:
            b = torch.empty(G, N, device=x.device)
            self._sample(lin, lin.mu_bias, lin.rho_bias, "bias", b, N, 1, 1, bias=True)
        y = torch.empty(G, rows, N, device=x.device)
        ops.conv2d_fwd(x, w, y, G, rows, 1, 1, K, N, 1, 1, 0, bias=b)
        return y, (lin, x, w, rows)

    def _linear_bwd(self, rec, dy, need_dx=True):
        lin, x, w, rows = rec
        G, N, K = self.G, lin.out_features, lin.in_features
        if lin.mu_weight.requires_grad:
            splits = ops.wgrad_splits(G, rows, 1, 1, K, N, 1, 1, 0)
            ws = torch.empty(splits, G, N, K, device=dy.device)
            ops.conv2d_bwd_weight(x, dy, ws, splits, G, rows, 1, 1, K, N, 1, 1, 0)
            self._reparam_bwd(lin, lin.mu_weight, lin.rho_weight, ws, splits, N, K, 1, "weight")
        if lin.mu_bias is not None and lin.mu_bias.requires_grad:
            db = torch.empty(G, N, device=dy.device)
            ops.colsum(dy, G, rows, N, db)
            self._reparam_bwd(lin, lin.mu_bias, lin.rho_bias, db, 1, N, 1, 1, "bias", bias=True)
        if not need_dx:
            return None
        dx = torch.empty(G, rows, K, device=dy.device)
        ops.conv2d_bwd_data(dy, w, dx, G, rows, 1, 1, K, N, 1, 1, 0)
        return dx


    # ---- AdditiveAttention (base_models.py:43-52): q|k|v as ONE GEMM over [Wq;Wk;Wv] ----
    @staticmethod
    def _att_dims(att):
        return att.query_projection.in_features, att.query_projection.out_features

    def _qkv(self, att, f, rows):
        G, dev = self.G, f.device
        D, Hd = self._att_dims(att)
        w = torch.empty(G, 3 * Hd, D, device=dev)
        b = torch.empty(G, 3 * Hd, device=dev)
        for j, lin in enumerate((att.query_projection, att.key_projection,
                                 att.value_projection)):
            self._sample(lin, lin.mu_weight, lin.rho_weight, "weight",
                         w.view(G, -1)[:, j * Hd * D:], Hd, D, 1, out_gstride=3 * Hd * D)
            self._sample(lin, lin.mu_bias, lin.rho_bias, "bias", b[:, j * Hd:], Hd, 1, 1,
                         bias=True, out_gstride=3 * Hd)
        qkv = torch.empty(G, rows, 3 * Hd, device=dev)
        ops.conv2d_fwd(f, w, qkv, G, rows, 1, 1, D, 3 * Hd, 1, 1, 0, bias=b)
        return qkv, w

    def _qkv_bwd(self, att, f, w, dqkv, rows, need_df=True):
        G, dev = self.G, dqkv.device
        D, Hd = self._att_dims(att)
        lins = (att.query_projection, att.key_projection, att.value_projection)
        if any(l.mu_weight.requires_grad for l in lins):
            splits = ops.wgrad_splits(G, rows, 1, 1, D, 3 * Hd, 1, 1, 0)
            ws = torch.empty(splits, G, 3 * Hd, D, device=dev)
            ops.conv2d_bwd_weight(f, dqkv, ws, splits, G, rows, 1, 1, D, 3 * Hd, 1, 1, 0)
            db = torch.empty(G, 3 * Hd, device=dev)
            ops.colsum(dqkv, G, rows, 3 * Hd, db)
            for j, lin in enumerate(lins):
                self._reparam_bwd(lin, lin.mu_weight, lin.rho_weight,
                                  ws.view(splits, G, -1)[:, :, j * Hd * D:], splits, Hd, D, 1,
                                  "weight", dw_gstride=3 * Hd * D, dw_sstride=G * 3 * Hd * D)
                self._reparam_bwd(lin, lin.mu_bias, lin.rho_bias, db[:, j * Hd:], 1, Hd, 1, 1,
                                  "bias", bias=True, dw_gstride=3 * Hd)
        if not need_df:
            return None
        df = torch.empty(G, rows, D, device=dev)
        ops.conv2d_bwd_data(dqkv, w, df, G, rows, 1, 1, D, 3 * Hd, 1, 1, 0)
        return df

    def _attention(self, att, f, rows, out, ld, off):
        """o = v * softmax(Wm tanh(q + k) + bm) into out[:, :, off:off+Hd] (row stride ld)."""
        Hd = self._att_dims(att)[1]
        qkv, wqkv = self._qkv(att, f, rows)
        t = torch.empty(self.G, rows, Hd, device=f.device)
        ops.attn_t(qkv, self.G * rows, Hd, t)
        s, rm_ = self._linear(att.attention_mechanism, t, rows)
        ops.attn_out(qkv, s, self.G * rows, Hd, out, ld, off)
        return (att, f, wqkv, qkv, t, s, rm_) if self.save else None

    def _attention_bwd(self, rec, dout, ld, off, rows, need_df=True):
        att, f, wqkv, qkv, t, s, rm_ = rec
        Hd = self._att_dims(att)[1]
        dqkv = torch.empty_like(qkv)
        ds = torch.empty_like(s)
        ops.attn_out_bwd(dout, ld, off, qkv, s, self.G * rows, Hd, dqkv, ds)
        dt = self._linear_bwd(rm_, ds)
        ops.attn_t_bwd(dt, t, self.G * rows, Hd, dqkv)
        return self._qkv_bwd(att, f, wqkv, dqkv, rows, need_df)


# ----------------------------------------------------------------------------- trunk
class _BN:
    """Saved state of one BatchNorm (+ReLU) for the backward."""
    __slots__ = ("bn", "y", "out", "stats", "relu", "M", "C", "batch_stats", "mask")

    def __init__(self, bn, y, out, stats, relu, M, C, batch_stats, mask=None):
        self.bn, self.y, self.out, self.stats, self.relu = bn, y, out, stats, relu
        self.M, self.C, self.batch_stats, self.mask = M, C, batch_stats, mask

    @property
    def scale(self):
        return self.stats[2]

    @property
    def shift(self):
        return self.stats[3]

    def lazy(self):
        """(scale, shift, relu) for a consumer that applies this BN on load."""
        return (self.stats[2], self.stats[3], int(self.relu))


class TrunkRunner(_Runner):
    """torchvision ResNet-50 trunk (Bayesian convs, train-mode BN) for G MC samples.

    Fusions (numerically the same BN/ReLU maths, fewer HBM passes):
    * BN statistics come from the producing conv's epilogue (per-m-tile Welford partials);
    * bn1/bn2 of every bottleneck are never materialised: conv2/conv3 apply
      relu(y*scale + shift) while loading their input (forward and weight-gradient), and their
      backward rebuilds the ReLU mask from y.
    """

    def __init__(self, trunk, state, G, sample0, save, dtype=torch.float32, join=None):
        super().__init__(state, G, sample0, save)
        self.trunk = trunk
        self.join = join  # caller's stream when this trunk runs on a stream of its own
        self.dt = dtype   # activation / sampled-weight storage (fp32, bf16 or f16)

    def _centre(self, bn):
        """The centre the 16-bit conv feeding ``bn`` stores its output around (CENTRE_Y): bn's
        running mean as of the last refresh_centres when bn normalises with batch statistics
        and tracks running ones, else None (fp32 storage, eval-mode BN, untracked statistics)."""
        if not CENTRE_Y or self.dt == torch.float32 or not bn.training or \
                not bn.track_running_stats or bn.running_mean is None:
            return None
        return self.st.centre(bn)

    def _cin_pad(self, Cin):
        """The convs move 16-byte channel chunks: input channels pad to 8 (16-bit) or 4 (fp32)
        (every conv after the stems has Cin % 64 == 0)."""
        q = 4 if self.dt == torch.float32 else 8
        return Cin if Cin % q == 0 else (Cin + q - 1) // q * q

    # ---- conv / bn units ----
    def _conv(self, conv, x, B, H, W, x_strides=None, x_bn=None, bn_stats=True, fold=None,
              ysh=None):
        """fold = (y3, scale, shift, res, res_bn, mask): x is the previous bottleneck's output,
        not yet materialised; this 1x1 conv forms it on load (ops.conv2d_fwd_fold; mask: its ReLU
        bits too) and self.fold_out holds it afterwards.  ysh: the stored output's centre
        (_centre of the BN it feeds)."""
        G, Cin, Cout, k = self.G, conv.in_channels, conv.out_channels, conv.kernel_size
        st, pd = conv.stride[0], conv.padding[0]
        cp = self._cin_pad(Cin)
        alloc = torch.zeros if cp != Cin else torch.empty
        dev = x.device if fold is None else fold[0].device
        w = alloc(G, Cout, k, k, cp, device=dev, dtype=self.dt)
        self._sample(conv, conv.mu_kernel, conv.rho_kernel, "kernel", w, Cout, Cin, k * k,
                     cin_pad=cp)
        Ho, Wo = ops.out_hw(H, k, st, pd), ops.out_hw(W, k, st, pd)
        y = torch.empty(G, B, Ho, Wo, Cout, device=dev, dtype=self.dt)
        part = None
        if bn_stats:
            nblk = ops.fwd_stat_blocks(G, B, H, W, Cin, Cout, k, st, pd)
            buf = torch.empty(2 * G * nblk * Cout + G * nblk, device=dev)
            part = (buf[:G * nblk * Cout], buf[G * nblk * Cout:2 * G * nblk * Cout],
                    buf[2 * G * nblk * Cout:], nblk)
        stats = None if part is None else part[:3]
        if fold is not None:
            y3, sc, sh, res, res_bn, mask = fold
            x = torch.empty_like(y3)
            if not ops.conv2d_fwd_fold(y3, sc, sh, res, res_bn, x, w, y, G, B, H, W, Cin, Cout,
                                       stats=stats, mask=mask, ysh=ysh):
                if mask is not None:
                    ops.bn_apply_mask(y3, sc, sh, res, x, mask, G, B * H * W, Cin, res_bn=res_bn)
                else:
                    ops.bn_apply(y3, sc, sh, res, 1, x, G, B * H * W, Cin, res_bn=res_bn)
                ops.conv2d_fwd(x, w, y, G, B, H, W, cp, Cout, k, st, pd, stats=stats, ysh=ysh)
            self.fold_out = x
        else:
            ops.conv2d_fwd(x, w, y, G, B, H, W, cp, Cout, k, st, pd, x_strides=x_strides,
                           x_bn=x_bn, stats=stats, alg_cin=Cin, ysh=ysh)
        rec = (conv, x, x_strides, x_bn, w, B, H, W) if self.save else None
        return y, rec, part

    @staticmethod
    def _masked_addend_ok(rec):
        """A 16-bit identity block's conv1 data gradient takes its residual addend under the
        block output's ReLU bits only in the pipelined kernel: Cout % 64 == 0 and every operand
        within its 31-bit buffer offsets (conv_pipe16_launch); otherwise dres is materialised."""
        conv, B, H, W = rec[0], rec[5], rec[6], rec[7]
        lim = 0x7fff0000 // 2
        return conv.out_channels % 64 == 0 and \
            B * H * W * max(conv.in_channels, conv.out_channels) <= lim

    def _fold_fits(self, conv, B, H, W):
        """conv (the next block's conv1) can form the block output on load: a 1x1 / stride-1
        conv with at least FOLD_MIN_TILES 256-row tiles in its launch."""
        if _first(conv.kernel_size) != 1 or _first(conv.stride) != 1 or _first(conv.padding) != 0:
            return False
        N = conv.out_channels
        tiles = -(-B * H * W // 256) * self.G * -(-N // (256 if N >= 256 else 128))
        return tiles >= FOLD_MIN_TILES

    def _dgrad_partials(self, rec, s):
        """fp32: a {p1, p2, nblk, y, ...} dict for conv2d_bwd_data(bn=...) — rec's data gradient
        is the output gradient of BN s — or None (16-bit, or the switch off)."""
        if not BWD_PARTIALS_F32 or self.dt != torch.float32 or s is None or \
                (s.out is not None and s.mask is None):
            return None
        conv, x, xs, x_bn, w, B, H, W = rec
        G, Cin, Cout, k = self.G, conv.in_channels, conv.out_channels, _first(conv.kernel_size)
        st, pd = _first(conv.stride), _first(conv.padding)
        nblk = ops.dgrad_stat_blocks(G, B, H, W, Cin, Cout, k, st, pd)
        buf = torch.empty(2, G, nblk, Cin, device=s.y.device)
        st_ = s.stats
        return dict(y=s.y, out=None, mask=s.mask, scale=st_[2], shift=st_[3], mean=st_[0],
                    invstd=st_[1], relu=int(s.relu), p1=buf[0], p2=buf[1], nblk=nblk)

    def _conv_bwd(self, rec, dy, need_dx=True, addend=None, dx=None, accumulate=False,
                  addend_mask=None, bn=None):
        """Weight gradient (+ reparameterisation backward) and data gradient (+ addend, counted
        only under addend_mask's ReLU bits when given)."""
        conv, x, xs, x_bn, w, B, H, W = rec
        G, Cin, Cout, k = self.G, conv.in_channels, conv.out_channels, conv.kernel_size
        st, pd = conv.stride[0], conv.padding[0]
        cp = self._cin_pad(Cin)
        if conv.mu_kernel.requires_grad:
            splits = ops.wgrad_splits(G, B, H, W, cp, Cout, k, st, pd)
            ws = torch.empty(splits, G, Cout, k * k * cp, device=dy.device)
            ops.conv2d_bwd_weight(x, dy, ws, splits, G, B, H, W, cp, Cout, k, st, pd,
                                  x_strides=xs, x_bn=x_bn, alg_cin=Cin)
            self._reparam_bwd(conv, conv.mu_kernel, conv.rho_kernel, ws, splits, Cout, Cin,
                              k * k, "kernel", dw_cin=cp)
            del ws
        if not need_dx:
            return None
        if dx is None:
            dx = torch.empty(G, B, H, W, Cin, device=dy.device, dtype=self.dt)
        ops.conv2d_bwd_data(dy, w, dx, G, B, H, W, Cin, Cout, k, st, pd, addend=addend,
                            accumulate=accumulate, addend_mask=addend_mask, bn=bn)
        return dx

    def _stem(self, conv, x, B, H, W, ysh=None):
        """conv1 over im2col rows of the images, shared by the G samples: one GEMM
        [M x Kp] . [Kp x G*Cout] (ops.stem_fwd); the sampled weights are the OIHW parameter
        rows [Cout][Cin*R*S] zero-padded to Kp."""
        G, Cin, Cout, k = self.G, conv.in_channels, conv.out_channels, conv.kernel_size
        st, pd = conv.stride[0], conv.padding[0]
        K = Cin * k * k
        Kp = ops.stem_kp(self.dt, K)
        Ho, Wo = ops.out_hw(H, k, st, pd), ops.out_hw(W, k, st, pd)
        M = B * Ho * Wo
        cols = torch.empty(M, Kp, device=x.device, dtype=self.dt)
        ops.stem_im2col(x, B, Cin, H, W, k, st, pd, Kp, cols)
        w = torch.zeros(G, Cout, Kp, device=x.device, dtype=self.dt)
        self._sample(conv, conv.mu_kernel, conv.rho_kernel, "kernel", w, Cout, K, 1, cin_pad=Kp)
        y = torch.empty(G, B, Ho, Wo, Cout, device=x.device, dtype=self.dt)
        nblk = ops.fwd_stat_blocks(G, B, H, W, Cin, Cout, k, st, pd)
        buf = torch.empty(2 * G * nblk * Cout + G * nblk, device=x.device)
        part = (buf[:G * nblk * Cout], buf[G * nblk * Cout:2 * G * nblk * Cout],
                buf[2 * G * nblk * Cout:], nblk)
        ops.stem_fwd(cols, w, y, G, M, Kp, Cout, part[:3], K, ysh=ysh)
        rec = ("stem", conv, cols, M, Kp) if self.save else None
        return y, rec, part

    def _stem_bwd(self, rec, dy):
        """Weight gradient of _stem: a 1x1 weight-gradient GEMM over the shared rows (group
        stride 0), then the reparameterisation backward over the [Cout][Kp] slabs."""
        _, conv, cols, M, Kp = rec
        if not conv.mu_kernel.requires_grad:
            return
        G, Cin, Cout, k = self.G, conv.in_channels, conv.out_channels, conv.kernel_size
        K = Cin * k * k
        xs = (0, Kp, Kp, Kp, 1)
        splits = ops.wgrad_splits(G, M, 1, 1, Kp, Cout, 1, 1, 0)
        ws = torch.empty(splits, G, Cout, Kp, device=dy.device)
        ops.conv2d_bwd_weight(cols, dy, ws, splits, G, M, 1, 1, Kp, Cout, 1, 1, 0, x_strides=xs,
                              alg_cin=K)
        self._reparam_bwd(conv, conv.mu_kernel, conv.rho_kernel, ws, splits, Cout, K, 1,
                          "kernel", dw_cin=Kp)

    def _bn(self, bn, y, part, relu, res=None, materialize=True, res_bn=None, ysh=None):
        """Statistics (from the conv epilogue partials) + optional materialised output.  ysh: the
        centre y was stored with (its conv's; the statistics then describe the stored values)."""
        G, C = self.G, y.shape[-1]
        M = y.numel() // (G * C)
        stats = torch.empty(4, G, C, device=y.device)
        mean, invstd, scale, shift = stats[0], stats[1], stats[2], stats[3]
        batch_stats = bn.training or not bn.track_running_stats
        if batch_stats:
            if bn.momentum is None:
                raise NotImplementedError("mauv: cumulative-average BN (momentum=None)")
            track = bn.training and bn.track_running_stats
            pm, pm2, pcnt, nblk = part
            ws = torch.empty(ops.bn_stats_workspace_floats(G, nblk, C), device=y.device)
            ops.bn_stats_finalize(G, nblk, C, pm, pm2, pcnt, bn.weight, bn.bias,
                                  bn.running_mean if track else None,
                                  bn.running_var if track else None, bn.momentum, bn.eps, ws,
                                  mean, invstd, scale, shift, ysh=ysh)
            if track:
                pending = getattr(self, "_nbt", None)
                if pending is None:
                    bn.num_batches_tracked.add_(G)
                else:   # one multi-tensor add per trunk forward (run_forward)
                    pending.append(bn.num_batches_tracked)
        else:
            if ysh is not None:
                raise RuntimeError("mauv: centred storage needs batch statistics (_centre)")
            ops.bn_eval_params(G, C, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                               bn.eps, scale, shift)
        out = mask = None
        if materialize:
            out = torch.empty_like(y)
            if relu and self.save and C <= 2048:
                mask = torch.empty(G * M * C // 8, dtype=torch.uint8, device=y.device)
                ops.bn_apply_mask(y, scale, shift, res, out, mask, G, M, C, res_bn=res_bn)
            else:
                ops.bn_apply(y, scale, shift, res, relu, out, G, M, C, res_bn=res_bn)
        rec = _BN(bn, y, out if relu and mask is None else None, stats, relu, M, C, batch_stats,
                  mask) if self.save else None
        self.last_lazy = (scale, shift, int(relu))  # for a consumer applying it on load
        return out, rec

    def _bn_bwd(self, rec, dout, want_dres=False, mask=None, pre=None):
        """mask: ReLU-mask bits applied to dout (a downsample BN fed the block output's
        dres = dout * mask without that tensor); pre: the partial sums dout's data gradient
        wrote (_dgrad_partials), so the partial pass is skipped."""
        if not rec.batch_stats:
            raise NotImplementedError("mauv: backward through eval-mode BN is not on the path "
                                      "(the reference trains and predicts in .train())")
        G, M, C, bn = self.G, rec.M, rec.C, rec.bn
        dy = torch.empty_like(rec.y)
        dres = torch.empty_like(rec.y) if want_dres else None
        ws = torch.empty(ops.bn_workspace_floats(G, M, C), device=dy.device)
        dg = bn.weight.grad if bn.weight.requires_grad else None
        db = bn.bias.grad if bn.bias.requires_grad else None
        s = rec.stats
        if pre is not None:
            ops.bn_bwd_ex(rec.y, None, rec.mask, dout, rec.relu, s[0], s[1], s[2], s[3], G, M, C,
                          ws, dy, dres, dg, db, pre=(pre["p1"], pre["p2"], pre["nblk"]))
        elif mask is not None:
            ops.bn_bwd_ex(rec.y, None, mask, dout, 1, s[0], s[1], s[2], s[3], G, M, C, ws, dy,
                          dres, dg, db)
        elif rec.mask is not None:
            ops.bn_bwd_mask(rec.y, rec.mask, dout, s[0], s[1], s[2], G, M, C, ws, dy, dres, dg, db)
        else:
            ops.bn_bwd(rec.y, rec.out, dout, rec.relu, s[0], s[1], s[2], G, M, C, ws, dy, dres,
                       dg, db, shift=s[3])
        return dy, dres

    # ---- schedule ----
    def run_forward(self, x):
        self._nbt = []
        try:
            return self._run_forward(x)
        finally:
            nbt, self._nbt = self._nbt, None
            if nbt:
                torch._foreach_add_(nbt, self.G)

    def _run_forward(self, x):
        t, G = self.trunk, self.G
        x = x.contiguous()
        if x.dtype != torch.float32:
            x = x.float()
        B, Cin, H, W = x.shape
        if Cin != t.conv1.in_channels:
            raise ValueError(f"trunk expects {t.conv1.in_channels} input channels, got {Cin}")
        self.B = B
        recs = self.recs = []
        c0 = self._centre(t.bn1)
        y, rc, part = self._stem(t.conv1, x, B, H, W, ysh=c0)
        H, W = y.shape[2], y.shape[3]
        Hp, Wp = ops.out_hw(H, 3, 2, 1), ops.out_hw(W, 3, 2, 1)
        p = torch.empty(G, B, Hp, Wp, 64, device=x.device, dtype=self.dt)
        idx = torch.empty(G, B, Hp, Wp, 64, dtype=torch.uint8, device=x.device) \
            if self.save else None
        # bn1 + relu applied inside the max-pool's loads
        _, rb = self._bn(t.bn1, y, part, relu=True, materialize=False, ysh=c0)
        scale, shift, _ = self.last_lazy
        ops.maxpool_fwd(y, G * B, H, W, 64, p, idx, bn=(scale, shift, G))
        del y, part
        self.stem = (rc, rb, idx, (H, W)) if self.save else None
        del idx
        cur, H, W = p, Hp, Wp
        blocks = list(t.blocks())
        # a 16-bit block output is formed by the next block's conv1 while it loads its tiles
        # (ops.conv2d_fwd_fold)
        fold_ok = FOLD and self.dt != torch.float32
        pend = None
        for i, blk in enumerate(blocks):
            c1, c2, c3 = (self._centre(b) for b in (blk.bn1, blk.bn2, blk.bn3))
            if pend is not None:
                y1, r1, p1 = self._conv(blk.conv1, None, B, H, W, fold=pend, ysh=c1)
                cur, pend, self.fold_out = self.fold_out, None, None
            else:
                y1, r1, p1 = self._conv(blk.conv1, cur, B, H, W, ysh=c1)
            _, s1 = self._bn(blk.bn1, y1, p1, relu=True, materialize=False, ysh=c1)
            y2, r2, p2 = self._conv(blk.conv2, y1, B, H, W, x_bn=self.last_lazy, ysh=c2)
            H2, W2 = y2.shape[2], y2.shape[3]
            _, s2 = self._bn(blk.bn2, y2, p2, relu=True, materialize=False, ysh=c2)
            y3, r3, p3 = self._conv(blk.conv3, y2, B, H2, W2, x_bn=self.last_lazy, ysh=c3)
            rd = sd = res_bn = None
            if blk.downsample is not None:   # its BN is applied inside bn3's residual add
                cd = self._centre(blk.downsample[1])
                res, rd, pd_ = self._conv(blk.downsample[0], cur, B, H, W, ysh=cd)
                _, sd = self._bn(blk.downsample[1], res, pd_, relu=False, materialize=False,
                                 ysh=cd)
                res_bn = self.last_lazy[:2]
            else:
                res = cur
            nxt = blocks[i + 1].conv1 if i + 1 < len(blocks) else None
            if fold_ok and nxt is not None and self._fold_fits(nxt, B, H2, W2):
                _, s3 = self._bn(blk.bn3, y3, p3, relu=True, materialize=False, ysh=c3)
                mask = None
                if self.save:   # the backward reads the block output's ReLU bits (_bn's rule)
                    mask = torch.empty(y3.numel() // 8, dtype=torch.uint8, device=y3.device)
                    s3.mask = mask
                pend = (y3,) + self.last_lazy[:2] + (res, res_bn, mask)
                a3 = None
            else:
                a3, s3 = self._bn(blk.bn3, y3, p3, relu=True, res=res, res_bn=res_bn, ysh=c3)
            del res
            if self.save:
                recs.append((r1, s1, r2, s2, r3, s3, rd, sd))
            else:
                del y1, y2, y3
            cur, H, W = a3, H2, W2
        self.final_hw = (H, W)
        feat = torch.empty(G, B, 2048, device=x.device)
        ops.avgpool_fwd(cur, G * B, H * W, 2048, feat)
        del cur
        if t.has_classifier():
            out, self.fc_rec = self._linear(t.fc, feat, B)
            if not self.save:
                self.fc_rec = None
            return out
        return feat

    def run_backward(self, dout):
        t, G, B = self.trunk, self.G, self.B
        self.st.grads(dout.device)
        if self.join is not None:   # dout comes from the fusion head's stream
            dout.record_stream(torch.cuda.current_stream())
        dout = dout.contiguous()
        if t.has_classifier():
            dfeat = self._linear_bwd(self.fc_rec, dout)
            self.fc_rec = None
        else:
            dfeat = dout
        H, W = self.final_hw
        da = torch.empty(G, B, H, W, 2048, device=dout.device, dtype=self.dt)
        ops.avgpool_bwd(dfeat, G * B, H * W, 2048, da)
        del dfeat
        pre3 = None   # the partials of this block's bn3, from the next block's conv1 data gradient
        while self.recs:
            r1, s1, r2, s2, r3, s3, rd, sd = self.recs.pop()
            # the residual gradient: dres = da * mask3, kept implicit when bn3 has mask bits
            rmask = s3.mask if RES_MASK and s3.mask is not None and \
                (rd is not None or self.dt == torch.float32 or self._masked_addend_ok(r1)) \
                else None
            dy3, dres = self._bn_bwd(s3, da, want_dres=rmask is None, pre=pre3)
            if rmask is not None:
                dres = da
            del da, s3, pre3
            pre2 = self._dgrad_partials(r3, s2)
            da2 = self._conv_bwd(r3, dy3, bn=pre2)
            del dy3, r3
            dy2, _ = self._bn_bwd(s2, da2, pre=pre2)
            del da2, s2, pre2
            pre1 = self._dgrad_partials(r2, s1)
            da1 = self._conv_bwd(r2, dy2, bn=pre1)
            del dy2, r2
            dy1, _ = self._bn_bwd(s1, da1, pre=pre1)
            del da1, s1, pre1
            pre3 = None
            if rd is not None:
                dyd, _ = self._bn_bwd(sd, dres, mask=rmask)
                del dres, sd
                dx = self._conv_bwd(r1, dy1)
                self._conv_bwd(rd, dyd, dx=dx, accumulate=True)
                del dyd, rd
            else:
                # dx is the previous block's block-output gradient: its bn3 partials come from
                # this epilogue (with its ReLU-mask bits), after the residual addend is added
                prev3 = self.recs[-1][5] if self.recs else None
                pre3 = self._dgrad_partials(r1, prev3) if prev3 is not None and \
                    prev3.mask is not None else None
                dx = self._conv_bwd(r1, dy1, addend=dres, addend_mask=rmask, bn=pre3)
                del dres
            del dy1, r1
            da = dx
        rc, rb, idx, (H, W) = self.stem
        self.stem = None
        da0 = torch.empty(G, B, H, W, 64, device=da.device, dtype=self.dt)
        ops.maxpool_bwd(da, idx, G * B, H, W, 64, da0)
        del da, idx
        dy0, _ = self._bn_bwd(rb, da0)
        del da0
        self._stem_bwd(rc, dy0)
        if self.st.grad_ready_hook is not None:
            self.st.grad_ready_hook(self.trunk)
        if self.join is not None:   # the caller's stream (optimizer, all-reduce) waits for us
            ev = torch.cuda.Event()
            ev.record()
            self.join.wait_event(ev)
        return (None,)


# ----------------------------------------------------------------------------- head
class HeadRunner(_Runner):
    """AdditiveAttention x3 + concat + fc -> fc1 -> fc2 (models/base_models.py:74-90)."""

    def __init__(self, model, state, G, sample0, save):
        super().__init__(state, G, sample0, save)
        self.m = model

    def run_forward(self, f_img, f_bathy, f_sss):
        m, G = self.m, self.G
        rows = f_img.shape[1]
        self.rows = rows
        atts = (m.attention_image, m.attention_bathy, m.attention_sss)
        widths = [self._att_dims(a)[1] for a in atts]
        ld = sum(widths)
        comb = torch.empty(G, rows, ld, device=f_img.device)
        self.att_recs = []
        off = 0
        for att, f, w in zip(atts, (f_img, f_bathy, f_sss), widths):
            self.att_recs.append((self._attention(att, f.contiguous(), rows, comb, ld, off),
                                  ld, off))
            off += w
        h1, self.r_fc = self._linear(m.fc, comb, rows)
        h2, self.r_fc1 = self._linear(m.fc1, h1, rows)
        out, self.r_fc2 = self._linear(m.fc2, h2, rows)
        if not self.save:
            self.r_fc = self.r_fc1 = self.r_fc2 = None
            self.att_recs = []
        return out

    def run_backward(self, dlogits):
        rows = self.rows
        self.st.grads(dlogits.device)
        dh2 = self._linear_bwd(self.r_fc2, dlogits.contiguous())
        dh1 = self._linear_bwd(self.r_fc1, dh2)
        dcomb = self._linear_bwd(self.r_fc, dh1)
        self.r_fc = self.r_fc1 = self.r_fc2 = None
        dfs = tuple(self._attention_bwd(rec, dcomb, ld, off, rows)
                    for rec, ld, off in self.att_recs)
        self.att_recs = []
        return dfs


class AttentionRunner(_Runner):
    """A standalone AdditiveAttention.forward (base_models.py:43-52) for G samples:
    [rows, d_model] -> [G, rows, hidden]."""

    def __init__(self, att, state, G, sample0, save):
        super().__init__(state, G, sample0, save)
        self.att = att

    def run_forward(self, f):
        self.shape = f.shape
        D, Hd = self._att_dims(self.att)
        if f.shape[-1] != D:
            raise ValueError(f"AdditiveAttention expects {D} features, got {f.shape[-1]}")
        rows = f.numel() // D
        self.rows = rows
        # every sample reads the same input: expand over the MC groups
        f3 = f.reshape(1, rows, D).float().expand(self.G, rows, D).contiguous()
        out = torch.empty(self.G, rows, Hd, device=f.device)
        self.rec = self._attention(self.att, f3, rows, out, Hd, 0)
        return out.reshape(self.G, *self.shape[:-1], Hd)

    def run_backward(self, dout):
        Hd = self._att_dims(self.att)[1]
        self.st.grads(dout.device)
        df = self._attention_bwd(self.rec, dout.reshape(self.G, self.rows, Hd).contiguous(),
                                 Hd, 0, self.rows)
        self.rec = None
        return (df.sum(0).reshape(self.shape),)


class LayerRunner(_Runner):
    """A standalone bayesian-torch layer (Conv2dReparameterization /
    LinearReparameterization.forward: w = mu + softplus(rho) eps, then F.conv2d / F.linear)
    for one MC sample, with its backward (dx, dmu, drho) — for layers called outside the
    compiled trunk / head schedules.  fp32, NCHW / [..., in_features] like the reference."""

    def __init__(self, layer, state, sample0, save):
        super().__init__(state, 1, sample0, save)
        self.m = layer

    def run_forward(self, x):
        m = self.m
        self.shape = x.shape
        if isinstance(m, LinearReparameterization):
            rows = x.numel() // m.in_features
            x3 = x.reshape(1, rows, m.in_features).float().contiguous()
            y, self.rec = self._linear(m, x3, rows)
            return y.reshape(*x.shape[:-1], m.out_features)
        B, C, H, W = x.shape
        x = x.float().contiguous()
        k, st, pd = m.kernel_size, m.stride[0], m.padding[0]
        w = torch.empty(1, m.out_channels, k, k, C, device=x.device)
        self._sample(m, m.mu_kernel, m.rho_kernel, "kernel", w, m.out_channels, C, k * k)
        bias = None
        if m.mu_bias is not None:
            bias = torch.empty(1, m.out_channels, device=x.device)
            self._sample(m, m.mu_bias, m.rho_bias, "bias", bias, m.out_channels, 1, 1, bias=True)
        Ho, Wo = ops.out_hw(H, k, st, pd), ops.out_hw(W, k, st, pd)
        y = torch.empty(1, B, Ho, Wo, m.out_channels, device=x.device)
        xs = (0, C * H * W, W, 1, H * W)   # the NCHW input read in place
        ops.conv2d_fwd(x, w, y, 1, B, H, W, C, m.out_channels, k, st, pd, bias=bias,
                       x_strides=xs)
        self.rec = (x, xs, w, (B, C, H, W, Ho, Wo)) if self.save else None
        return y[0].permute(0, 3, 1, 2)

    def run_backward(self, dy):
        m = self.m
        self.st.grads(dy.device)
        if isinstance(m, LinearReparameterization):
            dx = self._linear_bwd(self.rec, dy.reshape(1, -1, m.out_features).contiguous())
            self.rec = None
            return (dx.reshape(self.shape),)
        x, xs, w, (B, C, H, W, Ho, Wo) = self.rec
        self.rec = None
        k, st, pd, Co = m.kernel_size, m.stride[0], m.padding[0], m.out_channels
        dyh = dy.permute(0, 2, 3, 1).contiguous().float()   # NCHW grad -> NHWC
        if m.mu_kernel.requires_grad:
            splits = ops.wgrad_splits(1, B, H, W, C, Co, k, st, pd)
            ws = torch.empty(splits, 1, Co, k * k * C, device=dy.device)
            ops.conv2d_bwd_weight(x, dyh, ws, splits, 1, B, H, W, C, Co, k, st, pd,
                                  x_strides=xs)
            self._reparam_bwd(m, m.mu_kernel, m.rho_kernel, ws, splits, Co, C, k * k, "kernel")
        if m.mu_bias is not None and m.mu_bias.requires_grad:
            db = torch.empty(1, Co, device=dy.device)
            ops.colsum(dyh, 1, B * Ho * Wo, Co, db)
            self._reparam_bwd(m, m.mu_bias, m.rho_bias, db, 1, Co, 1, 1, "bias", bias=True)
        dx = torch.empty(1, B, H, W, C, device=dy.device)
        ops.conv2d_bwd_data(dyh, w, dx, 1, B, H, W, C, Co, k, st, pd)
        return (dx[0].permute(0, 3, 1, 2).contiguous(),)


# ----------------------------------------------------------------------------- entry points
def _check_trunk(trunk):
    from .resnet import ResNet
    if not isinstance(trunk, ResNet):
        raise TypeError(f"mauv engine needs a mauv.resnet.ResNet trunk, got {type(trunk)}")
    for m in (trunk.conv1,) + tuple(b.conv1 for b in trunk.blocks()):
        if not is_bayesian(m):
            raise TypeError("trunk is not Bayesian: convert it with dnn_to_bnn first "
                            "(models/model_utils.py:26-28,35)")


def _run(runner, params, inputs, save):
    if save:
        return _Engine.apply(runner, runner.st.anchor, *inputs)
    with torch.no_grad():
        return runner.run_forward(*inputs)


def _to_device(x, dev):
    return x if x.device == dev else x.to(dev, non_blocking=True)


def run_trunk_mc(trunk, x, num_mc, state=None, sample0=None, join=None):
    """[num_mc, B, 2048|C] for one ResNet trunk (root = the trunk unless ``state`` given)."""
    _check_trunk(trunk)
    st = state or root_state(trunk)
    dev = trunk.conv1.mu_kernel.device
    if dev.type != "cuda":
        raise RuntimeError("mauv: the model must be on a ROCm device (model.to('cuda'))")
    s0 = st.next_samples(num_mc) if sample0 is None else sample0
    params = st.plist(("trunk", id(trunk)), lambda: list(trunk.parameters()))
    save = needs_grad(params)
    runner = TrunkRunner(trunk, st, num_mc, s0, save, st.trunk_dtype(), join)
    x = _to_device(x, dev)
    if x.dtype != torch.float32:   # autocast callers may hand 16-bit images; stems read fp32
        x = x.float()
    return _run(runner, params, (x,), save)


def run_multimodal_mc(model, inputs, bathy, sss, num_mc):
    """[num_mc, B, C] logits of MultiModalModel for num_mc MC samples in one batched pass."""
    st = root_state(model)
    for trunk in (model.image_model_feat, model.bathy_model_feat, model.sss_model_feat):
        _check_trunk(trunk)
    dev = model.fc.mu_weight.device
    s0 = st.next_samples(num_mc)
    head_params = st.plist("head", lambda: [p for n, p in model.named_parameters()
                                            if not n.split(".")[0].endswith("_feat")])
    trunks = (model.image_model_feat, model.bathy_model_feat, model.sss_model_feat)
    xs = (inputs, bathy, sss)
    # Training only: concurrent trunks need the fusion head's backward to set up the gradient
    # arena first (it runs on the caller's stream before any trunk backward).  MC inference
    # keeps the trunks in sequence: its chunks are sized to fill HBM with one trunk's
    # activations (predict.mc_chunk), and three concurrent trunks measured +2 % at best while
    # tripling the peak (caching-allocator retries when HBM is already held: 5.3k vs 9.7k/s).
    if TRUNK_STREAMS and dev.type == "cuda" and torch.is_grad_enabled() \
            and needs_grad(head_params):
        cur = torch.cuda.current_stream(dev)
        feats = []
        for trunk, x, ts in zip(trunks, xs, _trunk_streams(dev)):
            ts.wait_stream(cur)
            if x.is_cuda:
                x.record_stream(ts)
            with torch.cuda.stream(ts):
                feats.append(run_trunk_mc(trunk, x, num_mc, st, s0, join=cur))
        for f, ts in zip(feats, _trunk_streams(dev)):
            cur.wait_stream(ts)
            f.record_stream(cur)
        f_img, f_bathy, f_sss = feats
    else:
        f_img, f_bathy, f_sss = (run_trunk_mc(t, x, num_mc, st, s0) for t, x in zip(trunks, xs))
    save = needs_grad(head_params) or any(f.requires_grad for f in (f_img, f_bathy, f_sss))
    runner = HeadRunner(model, st, num_mc, s0, save)
    return _run(runner, head_params, (f_img, f_bathy, f_sss), save)


def _standalone(module, runner_cls, x, *extra):
    st = root_state(module)
    dev = next(module.parameters()).device
    if dev.type != "cuda":
        raise RuntimeError("mauv: the layer must be on a ROCm device (module.to('cuda'))")
    params = list(module.parameters())
    save = needs_grad(params) or (torch.is_grad_enabled() and x.requires_grad)
    runner = runner_cls(module, st, *extra, save)
    return _run(runner, params, (_to_device(x, dev),), save)


def run_attention_mc(att, f, num_mc):
    """[num_mc, ..., hidden] of a standalone AdditiveAttention for num_mc MC samples."""
    s0 = root_state(att).next_samples(num_mc)
    return _standalone(att, AttentionRunner, f, num_mc, s0)


def run_layer(layer, x):
    """One stochastic forward of a standalone Bayesian conv / linear layer (differentiable)."""
    s0 = root_state(layer).next_samples(1)
    return _standalone(layer, LayerRunner, x, s0)
