"""Is the KL gradient added once?  get_kl_loss backward alone, then CE + KL, vs the oracle."""
import os
import sys

import torch

R = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "multimodal-auv_amd"))
from oracle import bayes_ref  # noqa: E402
from tests.helpers import build_pair  # noqa: E402
from mauv.kl import get_kl_loss  # noqa: E402
from mauv import mchead  # noqa: E402

o, m = build_pair(key="image_model")
(0.25 * get_kl_loss(m)).backward()
(0.25 * bayes_ref.get_kl_loss(o)).backward()
for n in ("model.fc.rho_weight", "model.layer4.2.conv2.rho_kernel", "model.conv1.mu_kernel"):
    a = dict(m.named_parameters())[n].grad.double().cpu().reshape(-1)
    b = dict(o.named_parameters())[n].grad.double().reshape(-1)
    print("KL only", n, "median ratio hip/oracle", (a / b).median().item())
for p in list(m.parameters()) + list(o.parameters()):
    p.grad = None
x = torch.randn(2, 3, 64, 64)
y = torch.tensor([1, 2])
lg = m.mc_forward(x.cuda(), 2)
ce, _, _ = mchead.mc_mean_ce(lg, y.cuda())
kl = get_kl_loss(m)
(ce + 0.25 * kl).backward()
g1 = {n: p.grad.double().cpu().clone() for n, p in m.named_parameters()}
for p in m.parameters():
    p.grad = None
lg = m.mc_forward(x.cuda(), 2)
ce, _, _ = mchead.mc_mean_ce(lg, y.cuda())
(ce + 0.0 * get_kl_loss(m)).backward()
g0 = {n: p.grad.double().cpu().clone() for n, p in m.named_parameters()}
for p in list(o.parameters()):
    p.grad = None
(0.25 * bayes_ref.get_kl_loss(o)).backward()
for n in ("model.fc.rho_weight", "model.layer4.2.conv2.rho_kernel", "model.conv1.mu_kernel"):
    kd = (g1[n] - g0[n]).reshape(-1)   # (not exact: different MC draws) -> use medians
    b = dict(o.named_parameters())[n].grad.double().reshape(-1)
    print("CE+KL minus CE", n, "median diff", kd.median().item(), "oracle KL median", b.median().item())
