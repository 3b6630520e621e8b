"""Diagnostic: 16-bit HIP gradients vs fp32 HIP gradients (same weights, same epsilons) at a
given resolution/batch — separates BN-backward conditioning from real defects.

    python tools/diag16.py S B N
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tests.golden.common import make_batches, SEED_DATA  # noqa: E402
from tests.helpers import build_pair, EpsBridge  # noqa: E402

S, B, N = (int(v) for v in sys.argv[1:4])
o, m = build_pair()
batch = make_batches(SEED_DATA, 1, B=B, S_opt=S, S_son=S)[0]
x, b, s, y = (t.cuda() for t in (batch["main_image"], batch["bathy_image"], batch["sss_image"],
                                 batch["label"]))
bridge = EpsBridge(o, m, 99)
with bridge, torch.no_grad():
    for _ in range(N):
        o(batch["main_image"][:1], batch["bathy_image"][:1], batch["sss_image"][:1])
bridge.collect()
from mauv.engine import root_state, set_precision  # noqa: E402
from mauv import mchead  # noqa: E402
root_state(m).eps_provider = bridge.provider


def grads(dt):
    set_precision(m, dt)
    for p in m.parameters():
        p.grad = None
    root_state(m).arena = None
    lg = m.mc_forward(x, b, s, N)
    mchead.mc_mean_ce(lg, y)[0].backward()
    return lg.detach(), {n: p.grad.detach().clone() for n, p in m.named_parameters()}


l32, g32 = grads(torch.float32)
for dt in (torch.bfloat16, torch.float16):
    l16, g16 = grads(dt)
    cos, rows = [], []
    for n, a in g16.items():
        t = g32[n]
        if t.norm() == 0:
            continue
        c = float((a.double().flatten() @ t.double().flatten()) /
                  (a.double().norm() * t.double().norm() + 1e-300))
        cos.append(c)
        rows.append((c, n))
    cos = np.array(cos)
    print(f"{dt}: logits max|d| {(l16 - l32).abs().max().item():.3e}  grad cosine vs fp32 HIP: "
          f"median {np.median(cos):.4f} p10 {np.quantile(cos, 0.1):.4f} min {cos.min():.4f}")
    for c, n in sorted(rows)[:6]:
        print(f"   worst {c:.4f} {n}")
    for key in ("fc2.mu_weight", "fc.mu_weight", "attention_image.query_projection.mu_weight",
                "image_model_feat.layer4.2.conv3.mu_kernel", "image_model_feat.layer4.2.bn3.weight",
                "image_model_feat.layer1.0.conv1.mu_kernel", "image_model_feat.conv1.mu_kernel",
                "image_model_feat.bn1.weight"):
        if key in g16:
            a, t = g16[key].double().flatten(), g32[key].double().flatten()
            print(f"   {key:55s} cos {float(a @ t / (a.norm() * t.norm() + 1e-300)):.4f} "
                  f"|g16|/|g32| {float(a.norm() / (t.norm() + 1e-300)):.3f}")
