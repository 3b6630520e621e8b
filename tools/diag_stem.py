"""Per-tensor gradient error of the unimodal model (64 px) vs the fp32 oracle and a float64
replay: the stem path under MAUV_STEM_GEMM (diagnostic)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "multimodal-auv_amd"))
from oracle import bayes_ref  # noqa: E402
from tests.golden.common import make_batches, SEED_DATA  # noqa: E402
from tests.helpers import build_pair, EpsBridge, oracle64  # noqa: E402
from mauv.engine import root_state  # noqa: E402
from mauv.kl import get_kl_loss  # noqa: E402
from mauv import mchead  # noqa: E402

o, m = build_pair(key="image_model")
import copy  # noqa: E402
o_pre = copy.deepcopy(o)
batch = make_batches(SEED_DATA, 1, B=2, S_opt=64, S_son=64)[0]
x, y = batch["main_image"], batch["label"]


def oracle_loss(model, dt=torch.float32):
    lg = torch.stack([model(x.to(dt)) for _ in range(2)])
    loss = F.cross_entropy(lg.mean(0), y) + 0.25 * bayes_ref.get_kl_loss(model) / 2
    loss.backward()
    return lg, loss


bridge = EpsBridge(o, m, 7)
with bridge:
    oracle_loss(o)
bridge.collect()
o64, _ = oracle64(o_pre, bridge.store, lambda mm: oracle_loss(mm, torch.float64))
root_state(m).eps_provider = bridge.provider
logits = m.mc_forward(x.cuda(), 2)
ce, _, _ = mchead.mc_mean_ce(logits, y.cuda())
(ce + 0.25 * get_kl_loss(m) / 2).backward()
rows = []
for (n, p), q, t in zip(m.named_parameters(), o.parameters(), o64.parameters()):
    if p.grad is None:
        rows.append((n, "none"))
        continue
    g, c, tt = p.grad.double().cpu(), q.grad.double(), t.grad.double()
    sc = tt.abs().max().item() + 1e-30
    rows.append((n, (g - tt).abs().max().item() / sc, (c - tt).abs().max().item() / sc,
                 int((torch.sign(g) != torch.sign(tt)).sum()), int((torch.sign(c) != torch.sign(tt)).sum()),
                 int((g == 0).sum()), int((tt == 0).sum())))
import numpy as np  # noqa: E402
print("STEM_GEMM", os.environ.get("MAUV_STEM_GEMM", "1"), "F32_MATH", os.environ.get("MAUV_F32_MATH"))
eh = np.array([r[1] for r in rows if r[1] != "none"])
ec = np.array([r[2] for r in rows if r[1] != "none"])
print("hip err median/90/max", np.median(eh), np.percentile(eh, 90), eh.max())
print("cpu err median/90/max", np.median(ec), np.percentile(ec, 90), ec.max())
for r in rows[:8]:
    print(r)
print("backward order (fc, layer4 ...):")
for r in rows[::-1][:40]:
    print(r)
worst = sorted([r for r in rows if r[1] != "none"], key=lambda r: -(r[1] / (r[2] + 1e-12)))[:8]
print("worst hip/cpu ratio:")
for r in worst:
    print(r)
