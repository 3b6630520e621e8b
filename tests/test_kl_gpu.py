"""get_kl_loss after parameters are re-bound in place (``p.data = ...``, bayesian-torch's own
MOPED idiom): the fused KL table must follow every mu / rho storage, not only the first
layer's (bayesian-torch 0.5.0 get_kl_loss, called at train/multimodal.py:114)."""
import pytest
import torch

from oracle import bayes_ref
from tests.helpers import build_pair

pytestmark = pytest.mark.gpu


def _rebind(model, gen):
    """Give two non-first layers fresh storages (new pointers, new values)."""
    conv = model.bathy_model_feat.layer2[1].conv2
    conv.rho_kernel.data = conv.rho_kernel.data.clone() - 2.0 * torch.rand(
        conv.rho_kernel.shape, generator=gen).to(conv.rho_kernel.device)
    fc1 = model.fc1
    fc1.mu_weight.data = fc1.mu_weight.data.clone() + 1.0 * torch.randn(
        fc1.mu_weight.shape, generator=gen).to(fc1.mu_weight.device)


def test_kl_follows_rebound_parameters():
    from mauv.kl import get_kl_loss
    o, m = build_pair()
    kl0 = get_kl_loss(m).item()          # builds and caches the pointer table
    assert abs(kl0 - bayes_ref.get_kl_loss(o).item()) <= 1e-5 * abs(kl0)
    _rebind(o, torch.Generator().manual_seed(3))
    _rebind(m, torch.Generator().manual_seed(3))
    torch.cuda.synchronize()
    ref = bayes_ref.get_kl_loss(o)
    kl = get_kl_loss(m)
    assert abs(kl.item() - kl0) > 1e-4 * abs(kl0)    # 10x the tolerance below: visible
    print(f"KL {kl0:.4f} -> {kl.item():.4f} (oracle {ref.item():.4f})")
    assert abs(kl.item() - ref.item()) <= 1e-5 * abs(ref.item()), (kl.item(), ref.item())
    # the backward writes dKL into the re-bound parameters' gradients
    ref.backward()
    kl.backward()
    for get in (lambda mm: mm.bathy_model_feat.layer2[1].conv2.rho_kernel,
                lambda mm: mm.fc1.mu_weight):
        g, gr = get(m).grad.double().cpu(), get(o).grad.double()
        err = ((g - gr).abs().max() / gr.abs().max()).item()
        assert err <= 1e-5, err
