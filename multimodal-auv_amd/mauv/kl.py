"""get_kl_loss — the KL term of the ELBO as ONE fused reduction over every Bayesian tensor.

Reference semantics (bayesian-torch 0.5.0 ``get_kl_loss``, called at train/multimodal.py:114,
:284 and train/unimodal.py:130,:262): ``sum over layers of [mean_w KL(q||p) + mean_b KL(q||p)]``
with q = N(mu, softplus(rho)^2), p = N(prior_mu, prior_sigma^2).  The reference walks 174
layers (~12 kernels each) and recomputes it for every MC sample although it does not depend
on the sample; here it is one two-kernel reduction (mauv_kl_fwd) with a fused backward
(mauv_kl_bwd) that adds dKL/dmu, dKL/drho straight into the gradient arena.
"""
import numpy as np
import torch

from . import ops
from .engine import root_state
from .layers import is_bayesian


def _entries(modules):
    out = []
    for m in modules:
        mu_w = m.mu_kernel if hasattr(m, "mu_kernel") else m.mu_weight
        rho_w = m.rho_kernel if hasattr(m, "rho_kernel") else m.rho_weight
        out.append((mu_w, rho_w, m.prior_mean, m.prior_variance))
        if m.mu_bias is not None:
            out.append((m.mu_bias, m.rho_bias, m.prior_mean, m.prior_variance))
    return out


class KLTable:
    def __init__(self, modules):
        self.entries = _entries(modules)
        self.n = len(self.entries)
        self.nmod = len(modules)
        self._fwd = None
        self._fwd_key = None
        self._bwd = None
        self._bwd_key = None

    def _build(self, with_grads, device):
        rows = np.zeros((self.n, 6), dtype=np.int64)
        for i, (mu, rho, pm, ps) in enumerate(self.entries):
            rows[i, 0] = mu.data_ptr()
            rows[i, 1] = rho.data_ptr()
            if with_grads:
                rows[i, 2] = mu.grad.data_ptr() if mu.grad is not None else 0
                rows[i, 3] = rho.grad.data_ptr() if rho.grad is not None else 0
            rows[i, 4] = mu.numel()
            rows[i, 5] = np.array([pm, ps], dtype=np.float32).view(np.int64)[0]
        return torch.from_numpy(rows).to(device)

    def _ptr_key(self):
        """Every mu / rho storage pointer: bayesian-torch's own MOPED idiom re-binds a layer's
        parameters with ``p.data = ...``, which moves that one tensor and no other."""
        return tuple(t.data_ptr() for e in self.entries for t in e[:2])

    def fwd_table(self, device):
        key = self._ptr_key()
        if self._fwd is None or self._fwd_key != key:
            self._fwd = self._build(False, device)
            self._fwd_key = key
        return self._fwd

    def bwd_table(self, device):
        key = self._ptr_key() + tuple((t.grad.data_ptr() if t.grad is not None else 0)
                                      for e in self.entries for t in e[:2])
        if self._bwd is None or self._bwd_key != key:
            for mu, rho, _, _ in self.entries:
                if mu.requires_grad and (mu.grad is None or rho.grad is None):
                    raise RuntimeError("KL backward: gradient arena not attached")
            self._bwd = self._build(True, device)
            self._bwd_key = key
        return self._bwd


def _kl_value(tab):
    dev = tab.entries[0][0].device
    out = torch.empty(1, device=dev)
    ws = torch.empty(tab.n * 32, dtype=torch.float64, device=dev)
    ops.kl_fwd(tab.fwd_table(dev), tab.n, ws, out)
    return out[0]


class _KL(torch.autograd.Function):
    @staticmethod
    def forward(ctx, owner, anchor):
        ctx.owner = owner
        return _kl_value(owner[0])

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g):
        tab, st = ctx.owner
        dev = tab.entries[0][0].device
        st.grads(dev)
        coef = g.reshape(1).float().contiguous()
        ops.kl_bwd(tab.bwd_table(dev), tab.n, coef)
        st.kl_bwd_count += 1
        if st.grad_ready_hook is not None:   # DistributedMC orders its slice all-reduces after it
            ev = torch.cuda.Event()
            ev.record()
            st.kl_bwd_event = ev
        return None, None


def kl_of_modules(modules, root=None):
    modules = [m for m in modules if is_bayesian(m)]
    dev = _entries(modules[:1])[0][0].device
    if dev.type != "cuda":
        raise RuntimeError("mauv get_kl_loss: the Bayesian layers live on the host; the KL "
                           "reduction runs in libmauv_hip on a ROCm device (model.to('cuda'))")
    owner_mod = root if root is not None else modules[0]
    key = "_mauv_kltab"
    tab = owner_mod.__dict__.get(key)
    if tab is None or tab.nmod != len(modules):
        tab = KLTable(modules)
        owner_mod.__dict__[key] = tab
    st = root_state(owner_mod)
    if torch.is_grad_enabled() and any(e[0].requires_grad for e in tab.entries):
        return _KL.apply((tab, st), st.anchor)
    with torch.no_grad():
        return _kl_value(tab)


def unwrap(model):
    while hasattr(model, "module") and isinstance(model.module, torch.nn.Module) and (
            isinstance(model, torch.nn.parallel.DistributedDataParallel) or
            isinstance(model, torch.nn.DataParallel) or getattr(model, "_mauv_wrapper", False)):
        model = model.module
    return model


def get_kl_loss(m):
    """Sum of every Bayesian layer's KL (bayesian-torch ``get_kl_loss`` semantics)."""
    m = unwrap(m)
    st = m.__dict__.get("_mauv_state")   # an engine model: its Bayesian layer list, built once
    bayes = st.plist("bayes", lambda: [x for x in m.modules() if is_bayesian(x)]) if st \
        else [x for x in m.modules() if is_bayesian(x)]
    if bayes:
        return kl_of_modules(bayes, root=m)
    kl = None  # foreign modules exposing kl_loss(): reference behaviour
    for layer in m.modules():
        if hasattr(layer, "kl_loss"):
            kl = layer.kl_loss() if kl is None else kl + layer.kl_loss()
    return kl
