"""Diagnostic: HIP fp32 gradients vs oracle fp32 and oracle fp64 ('truth') on one batch."""
import sys, os, copy
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd")]
import torch, torch.nn.functional as F
from oracle import bayes_ref
from tests.golden.common import make_batches, SEED_DATA
from tests.helpers import build_pair, EpsBridge, max_rel

S, B, N = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
o, m = build_pair()
o64 = copy.deepcopy(o).double()
batch = make_batches(SEED_DATA, 1, B=B, S_opt=S, S_son=S)[0]
x, b, s, y = batch["main_image"], batch["bathy_image"], batch["sss_image"], batch["label"]
bridge = EpsBridge(o, m, 99)
with bridge:
    ol = torch.stack([o(x, b, s) for _ in range(N)])
bridge.collect()
store = dict(bridge.store)
names64 = {id(mod): n for n, mod in o64.named_modules()}
cnt = {}
def src64(layer, name, shape):
    k = (names64[id(layer)], name); i = cnt.get(k, 0); cnt[k] = i + 1
    return store[k][i].double().reshape(shape)
bayes_ref.set_eps_source(src64)
ol64 = torch.stack([o64(x.double(), b.double(), s.double()) for _ in range(N)])
bayes_ref.set_eps_source(None)
(F.cross_entropy(ol.mean(0), y)).backward()
(F.cross_entropy(ol64.mean(0), y)).backward()
from mauv.engine import root_state
from mauv import mchead
root_state(m).eps_provider = bridge.provider
lg = m.mc_forward(x.cuda(), b.cuda(), s.cuda(), N)
mchead.mc_mean_ce(lg, y.cuda())[0].backward()
print("logits: hip-vs-64", max_rel(lg, ol64), " cpu32-vs-64", max_rel(ol, ol64))
rows = []
for (n, p32), p64, pm in zip(o.named_parameters(), o64.parameters(), m.parameters()):
    if p32.grad is None: continue
    rows.append((n, max_rel(pm.grad, p64.grad), max_rel(p32.grad, p64.grad)))
worst_h = sorted(rows, key=lambda r: -r[1])[:8]
print("worst hip-vs-64:")
for r in worst_h: print(f"  {r[0]:60s} hip {r[1]:.2e}  cpu32 {r[2]:.2e}")
import statistics
print("median hip", statistics.median(r[1] for r in rows), "median cpu32", statistics.median(r[2] for r in rows))
print("max hip", max(r[1] for r in rows), "max cpu32", max(r[2] for r in rows))
