"""Oracle: bayesian-torch 0.5.0 reparameterisation layers restated (TEST INFRASTRUCTURE ONLY).

bayesian-torch 0.5.0 is pinned by the reference (``pyproject.toml:41``,
``reqirements.txt:4``) but is neither installed nor vendored.  Call sites in the
reference: ``models/model_utils.py:6,26-28,35`` (``dnn_to_bnn``),
``train/multimodal.py:9,114,284`` and ``train/unimodal.py:9,130,262`` (``get_kl_loss``).
Restated from the library's published 0.5.0 algorithm:

* forward: ``sigma = log1p(exp(rho))``; ``eps ~ N(0,1)`` drawn fresh, weight-shaped, per
  forward call (shared by the whole batch); ``w = mu + sigma * eps`` (same for bias);
  then ``F.conv2d`` / ``F.linear``.  With ``dnn_to_bnn_flag`` set the layer returns only
  the output (no KL tuple).
* ``kl_div(mu_q, sigma_q, mu_p, sigma_p) = mean(log sigma_p - log sigma_q +
  (sigma_q^2 + (mu_q - mu_p)^2) / (2 sigma_p^2) - 1/2)``; a layer's ``kl_loss()`` sums the
  weight and bias terms; ``get_kl_loss(m)`` sums ``kl_loss()`` over ``m.modules()``.
* ``dnn_to_bnn`` (MOPED): recursive replacement of modules whose class name contains
  "Conv" / "Linear"; ``mu <- w``, ``rho <- log(expm1(delta * |w|) + 1e-20)``; prior
  ``mu_p = prior_mu``, ``sigma_p = prior_sigma`` (``prior_variance`` is used as a sigma).
* ``eps_*`` / ``prior_*`` buffers are non-persistent: the state_dict holds only
  ``mu_kernel, rho_kernel`` (conv) / ``mu_weight, rho_weight, mu_bias, rho_bias`` (linear).

Test hook: ``set_eps_source(fn)`` replaces the RNG draw with ``fn(layer, name, shape)``
so the HIP path and this oracle can be fed identical epsilons.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

_EPS_SOURCE = None


def set_eps_source(fn):
    """Install ``fn(layer, name, shape) -> Tensor`` as the epsilon source (None = RNG)."""
    global _EPS_SOURCE
    _EPS_SOURCE = fn


ALIAS_EPS = True   # bayesian-torch behaviour; False = fresh tensor per draw (exact gradient)


def _draw_eps(layer, name, buf):
    # bayesian-torch 0.5.0 does `eps = self.eps_kernel.data.normal_()`: the tensor autograd
    # saves for d(sigma*eps)/d(sigma) aliases the buffer, so when several MC forwards run
    # before one backward every pass's rho-gradient sees the LAST draw.  Reproduced here.
    if _EPS_SOURCE is None:
        e = buf.data.normal_()
        return e if ALIAS_EPS else e.clone()
    e = _EPS_SOURCE(layer, name, tuple(buf.shape))
    buf.data.copy_(e)
    return buf.data if ALIAS_EPS else e


def kl_div(mu_q, sigma_q, mu_p, sigma_p):
    kl = (torch.log(sigma_p) - torch.log(sigma_q)
          + (sigma_q ** 2 + (mu_q - mu_p) ** 2) / (2 * (sigma_p ** 2)) - 0.5)
    return kl.mean()


class Conv2dReparameterization(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0,
                 dilation=1, groups=1, prior_mean=0, prior_variance=1,
                 posterior_mu_init=0, posterior_rho_init=-3.0, bias=True):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride, self.padding = kernel_size, stride, padding
        self.dilation, self.groups = dilation, groups
        self.prior_mean, self.prior_variance = prior_mean, prior_variance
        self.posterior_mu_init, self.posterior_rho_init = posterior_mu_init, posterior_rho_init
        self.bias = bias
        self.dnn_to_bnn_flag = False
        shape = (out_channels, in_channels // groups, kernel_size, kernel_size)
        self.mu_kernel = nn.Parameter(torch.empty(shape))
        self.rho_kernel = nn.Parameter(torch.empty(shape))
        self.register_buffer("eps_kernel", torch.empty(shape), persistent=False)
        self.register_buffer("prior_weight_mu", torch.empty(shape), persistent=False)
        self.register_buffer("prior_weight_sigma", torch.empty(shape), persistent=False)
        if bias:
            self.mu_bias = nn.Parameter(torch.empty(out_channels))
            self.rho_bias = nn.Parameter(torch.empty(out_channels))
            self.register_buffer("eps_bias", torch.empty(out_channels), persistent=False)
            self.register_buffer("prior_bias_mu", torch.empty(out_channels), persistent=False)
            self.register_buffer("prior_bias_sigma", torch.empty(out_channels), persistent=False)
        else:
            self.register_parameter("mu_bias", None)
            self.register_parameter("rho_bias", None)
        self.init_parameters()

    def init_parameters(self):
        self.prior_weight_mu.fill_(self.prior_mean)
        self.prior_weight_sigma.fill_(self.prior_variance)
        self.mu_kernel.data.normal_(mean=self.posterior_mu_init, std=0.1)
        self.rho_kernel.data.normal_(mean=self.posterior_rho_init, std=0.1)
        if self.bias:
            self.prior_bias_mu.fill_(self.prior_mean)
            self.prior_bias_sigma.fill_(self.prior_variance)
            self.mu_bias.data.normal_(mean=self.posterior_mu_init, std=0.1)
            self.rho_bias.data.normal_(mean=self.posterior_rho_init, std=0.1)

    def kl_loss(self):
        sigma_weight = torch.log1p(torch.exp(self.rho_kernel))
        kl = kl_div(self.mu_kernel, sigma_weight, self.prior_weight_mu, self.prior_weight_sigma)
        if self.bias:
            sigma_bias = torch.log1p(torch.exp(self.rho_bias))
            kl = kl + kl_div(self.mu_bias, sigma_bias, self.prior_bias_mu, self.prior_bias_sigma)
        return kl

    def forward(self, input, return_kl=True):
        if self.dnn_to_bnn_flag:
            return_kl = False
        sigma_weight = torch.log1p(torch.exp(self.rho_kernel))
        eps_kernel = _draw_eps(self, "kernel", self.eps_kernel)
        weight = self.mu_kernel + sigma_weight * eps_kernel
        bias = None
        if self.bias:
            sigma_bias = torch.log1p(torch.exp(self.rho_bias))
            eps_bias = _draw_eps(self, "bias", self.eps_bias)
            bias = self.mu_bias + sigma_bias * eps_bias
        out = F.conv2d(input, weight, bias, self.stride, self.padding, self.dilation, self.groups)
        if return_kl:
            return out, self.kl_loss()
        return out


class LinearReparameterization(nn.Module):
    def __init__(self, in_features, out_features, prior_mean=0, prior_variance=1,
                 posterior_mu_init=0, posterior_rho_init=-3.0, bias=True):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.prior_mean, self.prior_variance = prior_mean, prior_variance
        self.posterior_mu_init, self.posterior_rho_init = posterior_mu_init, posterior_rho_init
        self.bias = bias
        self.dnn_to_bnn_flag = False
        shape = (out_features, in_features)
        self.mu_weight = nn.Parameter(torch.empty(shape))
        self.rho_weight = nn.Parameter(torch.empty(shape))
        self.register_buffer("eps_weight", torch.empty(shape), persistent=False)
        self.register_buffer("prior_weight_mu", torch.empty(shape), persistent=False)
        self.register_buffer("prior_weight_sigma", torch.empty(shape), persistent=False)
        if bias:
            self.mu_bias = nn.Parameter(torch.empty(out_features))
            self.rho_bias = nn.Parameter(torch.empty(out_features))
            self.register_buffer("eps_bias", torch.empty(out_features), persistent=False)
            self.register_buffer("prior_bias_mu", torch.empty(out_features), persistent=False)
            self.register_buffer("prior_bias_sigma", torch.empty(out_features), persistent=False)
        else:
            self.register_parameter("mu_bias", None)
            self.register_parameter("rho_bias", None)
        self.init_parameters()

    def init_parameters(self):
        self.prior_weight_mu.fill_(self.prior_mean)
        self.prior_weight_sigma.fill_(self.prior_variance)
        self.mu_weight.data.normal_(mean=self.posterior_mu_init, std=0.1)
        self.rho_weight.data.normal_(mean=self.posterior_rho_init, std=0.1)
        if self.bias:
            self.prior_bias_mu.fill_(self.prior_mean)
            self.prior_bias_sigma.fill_(self.prior_variance)
            self.mu_bias.data.normal_(mean=self.posterior_mu_init, std=0.1)
            self.rho_bias.data.normal_(mean=self.posterior_rho_init, std=0.1)

    def kl_loss(self):
        sigma_weight = torch.log1p(torch.exp(self.rho_weight))
        kl = kl_div(self.mu_weight, sigma_weight, self.prior_weight_mu, self.prior_weight_sigma)
        if self.bias:
            sigma_bias = torch.log1p(torch.exp(self.rho_bias))
            kl = kl + kl_div(self.mu_bias, sigma_bias, self.prior_bias_mu, self.prior_bias_sigma)
        return kl

    def forward(self, input, return_kl=True):
        if self.dnn_to_bnn_flag:
            return_kl = False
        sigma_weight = torch.log1p(torch.exp(self.rho_weight))
        eps_weight = _draw_eps(self, "weight", self.eps_weight)
        weight = self.mu_weight + sigma_weight * eps_weight
        bias = None
        if self.bias:
            sigma_bias = torch.log1p(torch.exp(self.rho_bias))
            eps_bias = _draw_eps(self, "bias", self.eps_bias)
            bias = self.mu_bias + sigma_bias * eps_bias
        out = F.linear(input, weight, bias)
        if return_kl:
            return out, self.kl_loss()
        return out


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
        layer.mu_kernel.data.copy_(d.weight.data)
        layer.rho_kernel.data.copy_(get_rho(d.weight.data, delta))
        if layer.mu_bias is not None:
            layer.mu_bias.data.copy_(d.bias.data)
            layer.rho_bias.data.copy_(get_rho(d.bias.data, delta))
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
        layer.mu_weight.data.copy_(d.weight.data)
        layer.rho_weight.data.copy_(get_rho(d.weight.data, delta))
        if layer.mu_bias is not None:
            layer.mu_bias.data.copy_(d.bias.data)
            layer.rho_bias.data.copy_(get_rho(d.bias.data, delta))
    layer.dnn_to_bnn_flag = True
    return layer


def dnn_to_bnn(m, bnn_prior_parameters):
    """In-place recursive Conv*/Linear* -> reparameterisation-layer conversion."""
    for name, value in list(m._modules.items()):
        if m._modules[name]._modules:
            dnn_to_bnn(m._modules[name], bnn_prior_parameters)
        elif "Conv" in m._modules[name].__class__.__name__:
            setattr(m, name, _bnn_conv_layer(bnn_prior_parameters, m._modules[name]))
        elif "Linear" in m._modules[name].__class__.__name__:
            setattr(m, name, _bnn_linear_layer(bnn_prior_parameters, m._modules[name]))
    return


def get_kl_loss(m):
    kl_loss = None
    for layer in m.modules():
        if hasattr(layer, "kl_loss"):
            if kl_loss is None:
                kl_loss = layer.kl_loss()
            else:
                kl_loss = kl_loss + layer.kl_loss()
    return kl_loss
