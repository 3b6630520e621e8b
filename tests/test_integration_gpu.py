"""INTEGRATION.md §2's ctypes snippet — the binding a reference-side maintainer would copy —
executed verbatim, and its output checked: each MC sample's weights are mu + softplus(rho) *
eps_g with eps_g ~ N(0, 1) (distinct per sample), and y[g] = conv(x[g], w[g]) (float64 torch,
1e-4 relative)."""
import os
import re

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_integration_snippet_runs_verbatim(monkeypatch):
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    sec = text[text.index("## 2."):]
    code = re.search(r"```python\n(.*?)```", sec, re.S).group(1)
    monkeypatch.chdir(REPO)
    ns = {}
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    x, w, y, mu, rho = (ns[k] for k in ("x", "w", "y", "mu", "rho"))
    G = ns["G"]
    # sampled weights: eps = (w - mu) / softplus(rho) is standard normal and differs per sample
    eps = (w.permute(0, 1, 4, 2, 3) - mu) / F.softplus(rho)
    assert abs(eps.mean().item()) < 0.02 and abs(eps.std().item() - 1) < 0.02
    assert not torch.equal(w[0], w[1])
    for g in range(G):
        ref = F.conv2d(x[g].permute(0, 3, 1, 2).double().cpu(),
                       w[g].permute(0, 3, 1, 2).double().cpu(), padding=1)
        got = y[g].permute(0, 3, 1, 2).double().cpu()
        assert (got - ref).abs().max().item() <= 1e-4 * ref.abs().max().item()
