"""Shared helpers for the parity tests: build matching oracle / mauv models and feed both the
same epsilons (the oracle's draws are recorded and replayed into the HIP sampler)."""
import torch

from oracle import bayes_ref
from oracle.model_ref import define_models as oracle_define, DEFAULT_PRIOR
from tests.golden.common import RecordingEpsSource


def build_pair(seed=0, num_classes=7, key="multimodal_model"):
    from mauv.models import define_models
    torch.manual_seed(seed)
    o = oracle_define(None, num_classes, DEFAULT_PRIOR)[key]
    torch.manual_seed(seed)
    m = define_models(None, num_classes, DEFAULT_PRIOR)[key]
    m.load_state_dict(o.state_dict())
    return o, m.cuda()


class EpsBridge:
    """Record the oracle's per-layer epsilons over N sequential passes and serve them to the
    mauv engine as [G, numel] tensors keyed by the same qualified module name."""

    def __init__(self, oracle_model, mauv_model, seed):
        self.src = RecordingEpsSource(seed)
        self.o_names = {id(mod): n for n, mod in oracle_model.named_modules()}
        self.m_names = {id(mod): n for n, mod in mauv_model.named_modules()}
        self.store = {}

    def __enter__(self):
        bayes_ref.set_eps_source(self.src)
        return self

    def __exit__(self, *a):
        bayes_ref.set_eps_source(None)

    def collect(self):
        self.store = {}
        for layer, name, e in self.src.log:
            self.store.setdefault((self.o_names[id(layer)], name), []).append(e.reshape(-1))
        self.src.log.clear()

    def provider(self, module, name, G):
        lst = self.store[(self.m_names[id(module)], name)]
        assert len(lst) >= G, (self.m_names[id(module)], name, len(lst), G)
        return torch.stack(lst[:G]).cuda().contiguous()

    def sequential(self):
        """A provider that hands out each layer's recorded draws in order across calls: MC
        chunks (mc_statistics with chunk < N) get passes 0..c-1, c..2c-1, ... as the oracle's
        sequential loop consumed them (``provider`` restarts at pass 0 on every call)."""
        used = {}

        def prov(module, name, G):
            k = (self.m_names[id(module)], name)
            i = used.get(k, 0)
            lst = self.store[k]
            assert len(lst) >= i + G, (k, len(lst), i, G)
            used[k] = i + G
            return torch.stack(lst[i:i + G]).cuda().contiguous()
        return prov


def oracle64(o, store, fn):
    """Run ``fn(o64)`` on a float64 copy of the oracle, replaying the recorded epsilons
    (``store`` from EpsBridge.collect) in the same per-layer order -> the 'truth' used to
    judge the fp32 HIP path against the fp32 CPU path (both are fp32 chains through an
    ill-conditioned BN backward at small spatial sizes)."""
    import copy
    o64 = copy.deepcopy(o).double()
    for p in o64.parameters():
        p.grad = None
    names = {id(mod): n for n, mod in o64.named_modules()}
    cnt = {}

    def src(layer, name, shape):
        k = (names[id(layer)], name)
        i = cnt.get(k, 0)
        cnt[k] = i + 1
        return store[k][i].double().reshape(shape)
    bayes_ref.set_eps_source(src)
    try:
        out = fn(o64)
    finally:
        bayes_ref.set_eps_source(None)
    return o64, out


def oracle_replay(o, store, fn, dtype=torch.float32, device="cpu"):
    """``fn(copy)`` on a copy of the oracle moved to ``device`` / ``dtype``, replaying the
    recorded epsilons (EpsBridge.collect) in the same per-layer order.  With device="cuda"
    and ``fn`` running under torch.autocast this is the reference's own mixed-precision
    scheme (inference/predictors.py:55) on the same weights and epsilons: the bar for the
    16-bit HIP paths."""
    import copy
    oc = copy.deepcopy(o).to(device=device, dtype=dtype)
    for p in oc.parameters():
        p.grad = None
    names = {id(mod): n for n, mod in oc.named_modules()}
    cnt = {}

    def src(layer, name, shape):
        k = (names[id(layer)], name)
        i = cnt.get(k, 0)
        cnt[k] = i + 1
        return store[k][i].to(dtype).reshape(shape)
    bayes_ref.set_eps_source(src)
    try:
        out = fn(oc)
    finally:
        bayes_ref.set_eps_source(None)
    return oc, out


def cosines(params, truth_params):
    """name -> cosine similarity of each parameter's gradient with the truth's gradient
    (tensors whose true gradient is zero are skipped)."""
    out = {}
    for (n, p), pt in zip(params, truth_params):
        if pt.grad is None or p.grad is None:
            continue
        t = pt.grad.detach().double().cpu().flatten()
        if t.norm() == 0:
            continue
        a = p.grad.detach().double().cpu().flatten()
        out[n] = float(a @ t / (a.norm() * t.norm() + 1e-300))
    return out


def fit_model(m, x, b, s, labels, steps=20, lr=1e-3, num_mc=2):
    """A few FusedAdam MC training steps (fp32) of a mauv model on one batch so that its
    predicted class depends on the input (tests of class agreement): at random init the
    per-item logits differ by ~3e-4 — less than the MC noise — and every item gets one class
    (every golden row is class 4).  Returns the cross-entropy of the last step."""
    from mauv.optim import FusedAdam
    from mauv.train import mc_train_step
    opt = FusedAdam(m.parameters(), lr=lr)
    crit = torch.nn.CrossEntropyLoss()
    ce = None
    for _ in range(steps):
        r = mc_train_step(m, (x, b, s), labels, crit, opt, num_mc, labels.numel(), 1e-6)
        ce = float(r["ce"])
    opt.zero_grad(set_to_none=True)
    return ce


def grad_error_profile(hip_params, cpu_params, truth_params):
    """Per-tensor max-relative errors of HIP and CPU-fp32 grads vs the fp64 truth."""
    hip, cpu = [], []
    for ph, pc, pt in zip(hip_params, cpu_params, truth_params):
        if pt.grad is None:
            continue
        hip.append(max_rel(ph.grad, pt.grad))
        cpu.append(max_rel(pc.grad, pt.grad))
    import numpy as np
    q = lambda v: np.quantile(np.array(v), [0.5, 0.9, 1.0])
    return q(hip), q(cpu)


def max_rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def forward_order(oracle_model, *inputs):
    """[(module name, eps name, shape)] in the order one oracle forward draws its epsilons —
    the order the reference's bayesian-torch layers consume torch's generator."""
    names = {id(mod): n for n, mod in oracle_model.named_modules()}
    order = []

    def src(layer, name, shape):
        order.append((names[id(layer)], name, shape))
        return torch.zeros(shape)
    bayes_ref.set_eps_source(src)
    try:
        with torch.no_grad():
            oracle_model(*inputs)
    finally:
        bayes_ref.set_eps_source(None)
    return order


class ReplayEps:
    """eps_provider for the mauv engine that replays ``eps_generator_source(seed)`` — the
    stream the golden run fed the reference — in the reference's consumption order: pass k of
    the sequential MC loop draws every layer's epsilon in forward order before pass k+1.  The
    engine asks per layer for the next G passes; each request that runs past the passes
    generated so far draws whole passes from the generator, so chunked MC consumption matches
    the sequential stream."""

    def __init__(self, model, order, seed):
        self.g = torch.Generator().manual_seed(seed)
        self.order = order
        self.names = {id(mod): n for n, mod in model.named_modules()}
        self.queues = {(n, e): [] for n, e, _ in order}

    def _draw_pass(self):
        for n, e, shape in self.order:
            self.queues[(n, e)].append(torch.randn(shape, generator=self.g).reshape(-1))

    def __call__(self, module, name, G):
        q = self.queues[(self.names[id(module)], name)]
        while len(q) < G:
            self._draw_pass()
        out, q[:G] = q[:G], []
        return torch.stack(out).cuda().contiguous()


class ListLoader:
    """Minimal DataLoader stand-in (iterable of batches with ``batch_size``), as the golden
    run fed the reference loops (tests/golden/make_golden.py)."""

    def __init__(self, batches, batch_size):
        self.batches, self.batch_size = batches, batch_size

    def __iter__(self):
        return iter(self.batches)

    def __len__(self):
        return len(self.batches)


class NullWriter:
    """SummaryWriter stand-in (tensorboard is not installed)."""

    def add_scalar(self, *a, **k):
        pass
