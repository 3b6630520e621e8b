"""bayesian-torch layer surface used on its own (the reference's ``bayesian_torch.layers``
and ``AdditiveAttention``, base_models.py:35-52): one stochastic forward through the HIP
sampler + implicit GEMM, differentiable through the engine's backward kernels.

Checked against float64 torch with the same injected epsilons: outputs and the gradients of
x, mu and rho (d/drho of softplus(rho) * eps = eps * sigmoid(rho)), within 1e-4 relative."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _close(a, ref, tol=1e-4):
    a, ref = a.detach().double().cpu(), ref.detach().double().cpu()
    d = (a - ref).abs().max().item()
    assert d <= tol * max(1.0, ref.abs().max().item()), d


class FixedEps:
    """eps_provider: one fixed N(0,1) tensor per (module, parameter) and MC sample."""

    def __init__(self, seed=0):
        self.g = torch.Generator().manual_seed(seed)
        self.store = {}

    def __call__(self, module, name, G):
        numel = (module.mu_kernel if name == "kernel" else
                 module.mu_weight if name == "weight" else module.mu_bias).numel()
        key = (id(module), name)
        if key not in self.store:
            self.store[key] = torch.randn(G, numel, generator=self.g)
        return self.store[key].to(DEV)

    def w(self, module, name, mu):
        return self.store[(id(module), name)][0].reshape(mu.shape).double()


def _sampled(p, rho, eps):
    return p.double() + F.softplus(rho.double()) * eps


def _install(layer):
    from mauv.engine import root_state
    prov = FixedEps(1)
    root_state(layer).eps_provider = prov
    return prov


@pytest.mark.parametrize("cin,cout,k,stride,pad,bias", [(3, 8, 3, 2, 1, True),
                                                        (16, 32, 1, 1, 0, False),
                                                        (1, 64, 7, 2, 3, False)])
def test_conv2d_reparameterization_forward_backward(cin, cout, k, stride, pad, bias):
    from bayesian_torch.layers import Conv2dReparameterization
    torch.manual_seed(0)
    layer = Conv2dReparameterization(cin, cout, k, stride=stride, padding=pad, bias=bias).to(DEV)
    prov = _install(layer)
    x = torch.randn(2, cin, 19, 19, device=DEV, requires_grad=True)
    out, kl = layer(x)
    b = _sampled(layer.mu_bias.cpu(), layer.rho_bias.cpu(),
                 prov.w(layer, "bias", layer.mu_bias)) if bias else None
    mu_r = layer.mu_kernel.detach().cpu().double().requires_grad_(True)
    rho_r = layer.rho_kernel.detach().cpu().double().requires_grad_(True)
    xr = x.detach().cpu().double().requires_grad_(True)
    wr = mu_r + F.softplus(rho_r) * prov.w(layer, "kernel", layer.mu_kernel)
    ref = F.conv2d(xr, wr, b, stride, pad)
    _close(out, ref)
    assert out.shape == ref.shape
    R = torch.randn(ref.shape, dtype=torch.float64)
    (ref * R).sum().backward()
    (out * R.to(DEV).float()).sum().backward()
    _close(x.grad, xr.grad)
    _close(layer.mu_kernel.grad, mu_r.grad)
    _close(layer.rho_kernel.grad, rho_r.grad)
    sig = F.softplus(layer.rho_kernel.detach().double().cpu())
    kl_ref = (-torch.log(sig) + (sig ** 2 + layer.mu_kernel.detach().double().cpu() ** 2) / 2
              - 0.5).mean()
    if bias:
        sb = F.softplus(layer.rho_bias.detach().double().cpu())
        kl_ref = kl_ref + (-torch.log(sb) + (sb ** 2 + layer.mu_bias.detach().double().cpu() ** 2)
                           / 2 - 0.5).mean()
    assert abs(kl.item() - kl_ref.item()) <= 1e-5 * abs(kl_ref.item())


@pytest.mark.parametrize("shape", [(5, 7), (2, 3, 7)])
def test_linear_reparameterization_forward_backward(shape):
    from bayesian_torch.layers import LinearReparameterization
    torch.manual_seed(1)
    layer = LinearReparameterization(7, 11).to(DEV)
    layer.dnn_to_bnn_flag = True        # returns the output only, as after dnn_to_bnn
    prov = _install(layer)
    x = torch.randn(*shape, device=DEV, requires_grad=True)
    out = layer(x)
    mu_r = layer.mu_weight.detach().cpu().double().requires_grad_(True)
    rho_r = layer.rho_weight.detach().cpu().double().requires_grad_(True)
    mub_r = layer.mu_bias.detach().cpu().double().requires_grad_(True)
    rhob_r = layer.rho_bias.detach().cpu().double().requires_grad_(True)
    xr = x.detach().cpu().double().requires_grad_(True)
    ref = F.linear(xr, mu_r + F.softplus(rho_r) * prov.w(layer, "weight", layer.mu_weight),
                   mub_r + F.softplus(rhob_r) * prov.w(layer, "bias", layer.mu_bias))
    _close(out, ref)
    R = torch.randn(ref.shape, dtype=torch.float64)
    (ref * R).sum().backward()
    (out * R.to(DEV).float()).sum().backward()
    for a, r in ((x, xr), (layer.mu_weight, mu_r), (layer.rho_weight, rho_r),
                 (layer.mu_bias, mub_r), (layer.rho_bias, rhob_r)):
        _close(a.grad, r.grad)


@pytest.mark.parametrize("d_model,hidden", [(2048, 128), (64, 32), (96, 200)])
def test_additive_attention_forward_backward(d_model, hidden):
    """AdditiveAttention.forward (base_models.py:43-52): keys/values/queries projections,
    tanh(q + k), softmax(Wm . + bm, dim=1), v * a — any d_model / hidden width."""
    from Multimodal_AUV.models.base_models import AdditiveAttention
    from mauv.layers import dnn_to_bnn
    from mauv.models import DEFAULT_PRIOR
    torch.manual_seed(2)
    att = AdditiveAttention(d_model, hidden_dim=hidden)
    dnn_to_bnn(att, DEFAULT_PRIOR)
    att = att.to(DEV)
    prov = _install(att)
    f = torch.randn(5, d_model, device=DEV, requires_grad=True)
    out = att(f)
    assert out.shape == (5, hidden)
    params = {}

    def lin(m, x):
        mw = m.mu_weight.detach().cpu().double().requires_grad_(True)
        rw = m.rho_weight.detach().cpu().double().requires_grad_(True)
        mb = m.mu_bias.detach().cpu().double().requires_grad_(True)
        rb = m.rho_bias.detach().cpu().double().requires_grad_(True)
        params[m] = (mw, rw, mb, rb)
        return F.linear(x, mw + F.softplus(rw) * prov.w(m, "weight", m.mu_weight),
                        mb + F.softplus(rb) * prov.w(m, "bias", m.mu_bias))
    fr = f.detach().cpu().double().requires_grad_(True)
    k = lin(att.key_projection, fr)
    v = lin(att.value_projection, fr)
    q = lin(att.query_projection, fr)
    a = torch.softmax(lin(att.attention_mechanism, torch.tanh(q + k)), dim=1)
    ref = v * a
    _close(out, ref)
    R = torch.randn(ref.shape, dtype=torch.float64)
    (ref * R).sum().backward()
    (out * R.to(DEV).float()).sum().backward()
    _close(f.grad, fr.grad)
    for m, (mw, rw, mb, rb) in params.items():
        _close(m.mu_weight.grad, mw.grad)
        _close(m.rho_weight.grad, rw.grad)
        _close(m.mu_bias.grad, mb.grad)
        _close(m.rho_bias.grad, rb.grad)
