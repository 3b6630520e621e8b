"""G9 diagnostic: parameters after the first Adam step of train_and_evaluate_unimodal_model on
the HIP path vs the oracle in fp32 and float64 (per-tensor count of elements whose update
differs from float64's by more than lr)."""
import copy
import os
import sys
import tempfile

import torch

R = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "multimodal-auv_amd"))
from oracle import bayes_ref, loops_ref  # noqa: E402
from oracle.model_ref import define_models as oracle_define, DEFAULT_PRIOR  # noqa: E402
from tests.golden.common import SEED_MODEL, SEED_EPS, SEED_DATA, make_batches, \
    eps_generator_source  # noqa: E402
from tests.helpers import forward_order, ReplayEps, ListLoader, NullWriter  # noqa: E402
from mauv.engine import root_state  # noqa: E402
import Multimodal_AUV.train.loop_utils as lu  # noqa: E402
from Multimodal_AUV.models.model_utils import define_models  # noqa: E402

DEV = torch.device("cuda")
LR = 5e-5
b = make_batches(SEED_DATA, 2, B=2, S_opt=64, S_son=64)
torch.manual_seed(SEED_MODEL)
o = oracle_define(None, 7, DEFAULT_PRIOR)
m = define_models(DEV, 7, DEFAULT_PRIOR)
keys = ("image_model", "bathy_model", "sss_model", "multimodal_model")
for k in keys:
    m[k].load_state_dict(o[k].state_dict())
    m[k] = m[k].to(DEV)
om = o["image_model"]
mm = m["image_model"]
root_state(mm).eps_provider = ReplayEps(mm, forward_order(copy.deepcopy(om), b[0]["main_image"]),
                                        SEED_EPS + 6)
crit, opts, schs = lu.define_optimizers_and_schedulers(
    m, {k: {"lr": LR} for k in keys}, {k: {"step_size": 1, "gamma": 0.5} for k in keys})
with tempfile.TemporaryDirectory() as d:
    import Multimodal_AUV.train.unimodal as um
    um.train_unimodal_model(mm, ListLoader(b[:1], 2), crit, opts["image_model"], epoch=1,
                            total_num_epochs=3, num_mc=2, sum_writer=NullWriter(), device=DEV,
                            model_type="image", csv_path=os.path.join(d, "x.csv"))


def oracle_step(dtype, rev=False):
    torch.manual_seed(SEED_MODEL)
    oo = oracle_define(None, 7, DEFAULT_PRIOR)["image_model"].to(dtype)
    opt = torch.optim.Adam(oo.parameters(), lr=LR)
    bayes_ref.set_eps_source(eps_generator_source(SEED_EPS + 6))
    xx, yy = b[0]["main_image"], b[0]["label"]
    if rev:
        xx, yy = xx.flip(0), yy.flip(0)
    try:
        r = loops_ref.train_step_unimodal(oo, xx.to(dtype), yy,
                                          torch.nn.CrossEntropyLoss(), opt, 1, 3, 2, 2)
    finally:
        bayes_ref.set_eps_source(None)
    return oo, r["loss"].item()


o32, l32 = oracle_step(torch.float32)
o64, l64 = oracle_step(torch.float64)
orv, _ = oracle_step(torch.float32, rev=True)
nrv = 0
for q, t, (n, p0) in zip(orv.parameters(), o64.parameters(), om.named_parameters()):
    nrv += int(((q.detach().double() - t.detach().double()).abs() > 0.5 * LR).sum())
print("reversed-batch cpu fp32 update differs from fp64:", nrv)
print("step loss fp32", l32, "fp64", l64)
init = dict(om.named_parameters())
rows = []
tot = [0, 0, 0]
for (n, p), q, t in zip(mm.named_parameters(), o32.parameters(), o64.parameters()):
    p0 = init[n].double()
    ug = p.detach().double().cpu() - p0
    uc = q.detach().double() - p0
    ut = t.detach().double() - p0
    fg = int(((ug - ut).abs() > 0.5 * LR).sum())
    fc = int(((uc - ut).abs() > 0.5 * LR).sum())
    z = int((ug.abs() < 0.5 * LR).sum())
    tot[0] += fg
    tot[1] += fc
    tot[2] += p.numel()
    rows.append((n, p.numel(), fg, fc, z, int((ut.abs() < 0.5 * LR).sum())))
print("total elements", tot[2], "update differs from fp64: hip", tot[0], "cpu fp32", tot[1])
print("(name, numel, hip_diff, cpu_diff, hip_zero_updates, fp64_zero_updates)")
for r in sorted(rows, key=lambda r: -(r[2] - r[3]))[:12]:
    print(r)
for r in rows[:6]:
    print(r)
name = "model.layer4.2.conv2.rho_kernel"
pm = dict(mm.named_parameters())[name]
pc = dict(o32.named_parameters())[name]
pt = dict(o64.named_parameters())[name]
p0 = init[name].double()
ug = (pm.detach().double().cpu() - p0).reshape(-1)
uc = (pc.detach().double() - p0).reshape(-1)
ut = (pt.detach().double() - p0).reshape(-1)
gg = pm.grad.double().cpu().reshape(-1) if pm.grad is not None else None
gc = pc.grad.double().reshape(-1)
gt = pt.grad.double().reshape(-1)
bad = ((ug - ut).abs() > 0.5 * LR).nonzero().reshape(-1)[:12]
print("elements where the HIP update differs (update hip/cpu/fp64 in units of lr; grads):")
for i in bad.tolist():
    print(i, round(ug[i].item() / LR, 3), round(uc[i].item() / LR, 3), round(ut[i].item() / LR, 3),
          None if gg is None else f"{gg[i].item():.3e}", f"{gc[i].item():.3e}", f"{gt[i].item():.3e}")
print("grad abs median hip/cpu/fp64", None if gg is None else gg.abs().median().item(), gc.abs().median().item(), gt.abs().median().item())
print("max |g_hip-g64|", None if gg is None else (gg - gt).abs().max().item(), "max |g_cpu-g64|", (gc - gt).abs().max().item())
d_h = gg - gt
d_c = gc - gt
print("median(g_hip - g64)", d_h.median().item(), "median(g_cpu - g64)", d_c.median().item())
rho0 = init[name].detach().double().reshape(-1)
s = torch.nn.functional.softplus(rho0)
mod = dict(om.named_modules())[name.rsplit(".", 1)[0]]
sp = float(mod.prior_variance)
klg = (-1.0 / s + s / sp ** 2) * torch.sigmoid(rho0) * (0.5 / 2 / rho0.numel())
print("analytic KL part of drho: median", klg.median().item(), "prior sigma", sp)
for nm in ("model.fc.rho_weight", "model.layer4.2.bn3.weight", "model.conv1.rho_kernel", "model.layer1.0.conv1.rho_kernel"):
    a = dict(mm.named_parameters())[nm].grad.double().cpu().reshape(-1)
    t = dict(o64.named_parameters())[nm].grad.double().reshape(-1)
    c = dict(o32.named_parameters())[nm].grad.double().reshape(-1)
    print(nm, "median hip-64", (a - t).median().item(), "cpu-64", (c - t).median().item(), "median|g64|", t.abs().median().item())
