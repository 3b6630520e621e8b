"""Bayesian layer modules with bayesian-torch 0.5.0's parameter surface.

``Conv2dReparameterization`` / ``LinearReparameterization`` keep the exact parameter names
and shapes the reference's checkpoints use (``mu_kernel, rho_kernel`` OIHW;
``mu_weight, rho_weight, mu_bias, rho_bias``) so ``state_dict`` / ``load_state_dict`` are
interchangeable with the reference.  Inside the models they are
parameter holders: the MC-batched engine (``mauv.engine``) samples and consumes them inside
HIP kernels.  A layer's own ``forward`` runs one sample through the same kernels, with the
engine's backward (``engine.LayerRunner``).

``dnn_to_bnn`` mirrors bayesian-torch's MOPED conversion used at
``models/model_utils.py:26-28,35`` (mu <- w, rho <- log(expm1(delta*|w|) + 1e-20)).
"""
import math

import torch
import torch.nn as nn



def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


class _BayesBase(nn.Module):
    # prior sigma/mean are scalars (bayesian-torch fills weight-shaped non-persistent buffers
    # with these constants; nothing else reads them, so no per-element buffers are kept)
    def _init_prior(self, prior_mean, prior_variance, posterior_mu_init, posterior_rho_init):
        self.prior_mean = float(prior_mean)
        self.prior_variance = float(prior_variance)
        self.posterior_mu_init = float(posterior_mu_init)
        self.posterior_rho_init = float(posterior_rho_init)
        self.dnn_to_bnn_flag = False

    def init_parameters(self):
        with torch.no_grad():
            self._mu().normal_(self.posterior_mu_init, 0.1)
            self._rho().normal_(self.posterior_rho_init, 0.1)
            if self.mu_bias is not None:
                self.mu_bias.normal_(self.posterior_mu_init, 0.1)
                self.rho_bias.normal_(self.posterior_rho_init, 0.1)

    def kl_loss(self):
        from .kl import kl_of_modules
        return kl_of_modules([self])


class Conv2dReparameterization(_BayesBase):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, prior_mean=0, prior_variance=1, posterior_mu_init=0,
                 posterior_rho_init=-3.0, bias=True):
        super().__init__()
        if groups != 1 or _pair(dilation) != (1, 1):
            raise NotImplementedError("mauv: grouped / dilated Bayesian convs are not on the path")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size = kernel_size if isinstance(kernel_size, int) else kernel_size[0]
        self.stride, self.padding = _pair(stride), _pair(padding)
        self.dilation, self.groups = _pair(dilation), groups
        self.bias = bias
        self._init_prior(prior_mean, prior_variance, posterior_mu_init, posterior_rho_init)
        k = self.kernel_size
        self.mu_kernel = nn.Parameter(torch.empty(out_channels, in_channels, k, k))
        self.rho_kernel = nn.Parameter(torch.empty(out_channels, in_channels, k, k))
        if bias:
            self.mu_bias = nn.Parameter(torch.empty(out_channels))
            self.rho_bias = nn.Parameter(torch.empty(out_channels))
        else:
            self.register_parameter("mu_bias", None)
            self.register_parameter("rho_bias", None)
        self.init_parameters()

    def _mu(self):
        return self.mu_kernel

    def _rho(self):
        return self.rho_kernel

    def extra_repr(self):
        return (f"{self.in_channels}, {self.out_channels}, kernel_size={self.kernel_size}, "
                f"stride={self.stride}, padding={self.padding}, bias={self.bias}")

    def forward(self, x, return_kl=True):
        """One MC sample (bayesian-torch Conv2dReparameterization.forward): w = mu +
        softplus(rho) * eps, F.conv2d — NCHW in / out through the HIP sampler and implicit
        GEMM, differentiable (dx, dmu, drho by the engine's backward kernels)."""
        from .engine import run_layer
        out = run_layer(self, x)
        if return_kl and not self.dnn_to_bnn_flag:
            return out, self.kl_loss()
        return out


class LinearReparameterization(_BayesBase):
    def __init__(self, in_features, out_features, prior_mean=0, prior_variance=1,
                 posterior_mu_init=0, posterior_rho_init=-3.0, bias=True):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.bias = bias
        self._init_prior(prior_mean, prior_variance, posterior_mu_init, posterior_rho_init)
        self.mu_weight = nn.Parameter(torch.empty(out_features, in_features))
        self.rho_weight = nn.Parameter(torch.empty(out_features, in_features))
        if bias:
            self.mu_bias = nn.Parameter(torch.empty(out_features))
            self.rho_bias = nn.Parameter(torch.empty(out_features))
        else:
            self.register_parameter("mu_bias", None)
            self.register_parameter("rho_bias", None)
        self.init_parameters()

    def _mu(self):
        return self.mu_weight

    def _rho(self):
        return self.rho_weight

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, bias={self.bias}"

    def forward(self, x, return_kl=True):
        """One MC sample (bayesian-torch LinearReparameterization.forward): w = mu +
        softplus(rho) * eps, F.linear over the last dim, through the HIP GEMM (differentiable)."""
        from .engine import run_layer
        out = run_layer(self, x)
        if return_kl and not self.dnn_to_bnn_flag:
            return out, self.kl_loss()
        return out


def is_bayesian(m):
    return isinstance(m, (Conv2dReparameterization, LinearReparameterization))


def get_rho(sigma, delta):
    return torch.log(torch.expm1(delta * torch.abs(sigma)) + 1e-20)


def _bnn_conv_layer(params, d):
    layer = Conv2dReparameterization(
        in_channels=d.in_channels, out_channels=d.out_channels, kernel_size=d.kernel_size[0],
        stride=d.stride, padding=d.padding, dilation=d.dilation, groups=d.groups,
        prior_mean=params["prior_mu"], prior_variance=params["prior_sigma"],
        posterior_mu_init=params["posterior_mu_init"],
        posterior_rho_init=params["posterior_rho_init"], bias=d.bias is not None)
    if params.get("moped_enable", False):
        delta = params["moped_delta"]
        with torch.no_grad():
            layer.mu_kernel.copy_(d.weight)
            layer.rho_kernel.copy_(get_rho(d.weight, delta))
            if layer.mu_bias is not None:
                layer.mu_bias.copy_(d.bias)
                layer.rho_bias.copy_(get_rho(d.bias, delta))
    layer.dnn_to_bnn_flag = True
    return layer


def _bnn_linear_layer(params, d):
    layer = LinearReparameterization(
        in_features=d.in_features, out_features=d.out_features,
        prior_mean=params["prior_mu"], prior_variance=params["prior_sigma"],
        posterior_mu_init=params["posterior_mu_init"],
        posterior_rho_init=params["posterior_rho_init"], bias=d.bias is not None)
    if params.get("moped_enable", False):
        delta = params["moped_delta"]
        with torch.no_grad():
            layer.mu_weight.copy_(d.weight)
            layer.rho_weight.copy_(get_rho(d.weight, delta))
            if layer.mu_bias is not None:
                layer.mu_bias.copy_(d.bias)
                layer.rho_bias.copy_(get_rho(d.bias, delta))
    layer.dnn_to_bnn_flag = True
    return layer


def dnn_to_bnn(m, bnn_prior_parameters):
    """In-place Conv*/Linear* -> reparameterisation layers (bayesian-torch 0.5.0 semantics)."""
    for name in list(m._modules):
        child = m._modules[name]
        if child is None:
            continue
        if child._modules:
            dnn_to_bnn(child, bnn_prior_parameters)
        elif "Conv" in child.__class__.__name__ and not is_bayesian(child):
            setattr(m, name, _bnn_conv_layer(bnn_prior_parameters, child))
        elif "Linear" in child.__class__.__name__ and not is_bayesian(child):
            setattr(m, name, _bnn_linear_layer(bnn_prior_parameters, child))
    m.__dict__.pop("_mauv_state", None)  # engine plan / layer ids change with the structure
