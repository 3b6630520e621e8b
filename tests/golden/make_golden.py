"""Generate golden vectors by running the REFERENCE's own Python (run in the survey container).

The reference (sams-tom/Multimodal-AUV, read-only at /root/reference) imports torchvision,
bayesian_torch and torch.utils.tensorboard, none of which are installed.  This script
installs the oracle's restatements of those third-party pieces as the modules the
reference imports (``torchvision.models`` -> ``oracle.resnet_ref``,
``bayesian_torch.models.dnn_to_bnn`` -> ``oracle.bayes_ref``; SummaryWriter -> a no-op
stub), bypasses ``Multimodal_AUV/__init__.py`` (it pulls in HF-hub/Examples), and then
drives the reference's OWN code:

  G3  models/model_utils.py:define_models + base_models.py:MultiModalModel.forward
      (MC logits at 64x64, B=2, N=3, injected epsilons)
  G5  train/multimodal.py:train_multimodal_model   (one epoch, 2 batches, num_mc=2)
  G6  train/multimodal.py:evaluate_multimodal_model + inference/predictors.py:
      multimodal_predict_and_save (CSV rows)
  G7  train/unimodal.py:train_unimodal_model (ResNet50Custom BNN, config 1 path, 64x64)
  G8  train/loop_utils.py:train_and_evaluate_multimodal_model (epoch driver, 2 epochs)
  G9  train/loop_utils.py:train_and_evaluate_unimodal_model (epoch driver, range(1, 3))
      (``--loops``: writes golden_loops.json only)
  G10 Examples/"Example training with image noise.py":simulate_underwater_degradation
      (``--staging``: writes golden_staging.npz only)

Epsilons come from one seeded torch.Generator consumed in forward order, so the oracle
(``oracle/``) reproduces them by running the same module order.  Outputs land in
``tests/golden/golden.json`` + ``golden.npz`` (small: logits, losses, uncertainty vectors,
a few parameter slices and checksums).  Re-run: ``python tests/golden/make_golden.py``.
"""
import csv
import importlib
import json
import os
import sys
import tempfile
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF_PKG = "/root/reference/src/Multimodal_AUV"
sys.path.insert(0, REPO)

from oracle import resnet_ref, bayes_ref  # noqa: E402
from tests.golden.common import (SEED_MODEL, SEED_EPS, SEED_DATA, make_batches,  # noqa: E402
                                 eps_generator_source, param_digest)


def install_shims():
    tv = types.ModuleType("torchvision")
    tvm = types.ModuleType("torchvision.models")
    tvm.resnet50 = resnet_ref.resnet50
    tvm.ResNet50_Weights = resnet_ref.ResNet50_Weights
    tv.models = tvm
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.models"] = tvm
    bt = types.ModuleType("bayesian_torch")
    btm = types.ModuleType("bayesian_torch.models")
    btd = types.ModuleType("bayesian_torch.models.dnn_to_bnn")
    btd.dnn_to_bnn = bayes_ref.dnn_to_bnn
    btd.get_kl_loss = bayes_ref.get_kl_loss
    sys.modules["bayesian_torch"] = bt
    sys.modules["bayesian_torch.models"] = btm
    sys.modules["bayesian_torch.models.dnn_to_bnn"] = btd
    tb = types.ModuleType("torch.utils.tensorboard")

    class SummaryWriter:
        def __init__(self, *a, **k):
            pass

        def add_scalar(self, *a, **k):
            pass

    tb.SummaryWriter = SummaryWriter
    sys.modules["torch.utils.tensorboard"] = tb
    pkg = types.ModuleType("Multimodal_AUV")
    pkg.__path__ = [REF_PKG]
    sys.modules["Multimodal_AUV"] = pkg
    return SummaryWriter


class ListLoader:
    """Minimal DataLoader stand-in: iterable of batch dicts with ``batch_size``."""

    def __init__(self, batches, batch_size):
        self.batches, self.batch_size = batches, batch_size

    def __iter__(self):
        return iter(self.batches)

    def __len__(self):
        return len(self.batches)


def main():
    SummaryWriter = install_shims()
    mu = importlib.import_module("Multimodal_AUV.models.model_utils")
    mm = importlib.import_module("Multimodal_AUV.train.multimodal")
    um = importlib.import_module("Multimodal_AUV.train.unimodal")
    pr = importlib.import_module("Multimodal_AUV.inference.predictors")
    prior = {"prior_mu": 0.0, "prior_sigma": 1.0, "posterior_mu_init": 0.0,
             "posterior_rho_init": -3.0, "type": "Reparameterization",
             "moped_enable": True, "moped_delta": 0.1}
    out, arrays = {}, {}
    tmp = tempfile.mkdtemp()
    torch.set_num_threads(8)
    here = os.path.dirname(os.path.abspath(__file__))
    if "--staging" in sys.argv:   # G10 only (golden_staging.npz)
        staging_golden(here)
        return
    if "--loops" in sys.argv:   # G8/G9 only (golden_loops.json); G3-G7 stay as committed
        loops_golden(mu, SummaryWriter, prior, tmp, here)
        return

    # ---------------- G3: reference define_models + MultiModalModel forward -------------
    torch.manual_seed(SEED_MODEL)
    models = mu.define_models(torch.device("cpu"), 7, prior)
    model = models["multimodal_model"]
    batches = make_batches(SEED_DATA, n_batches=2, B=2, S_opt=64, S_son=64)
    b0 = batches[0]
    bayes_ref.set_eps_source(eps_generator_source(SEED_EPS))
    model.train()
    with torch.no_grad():
        logits = torch.stack([model(b0["main_image"], b0["bathy_image"], b0["sss_image"])
                              for _ in range(3)])
    arrays["g3_logits"] = logits.numpy()
    out["g3_kl"] = float(bayes_ref.get_kl_loss(model).detach())
    out["g3_param_digest"] = param_digest(model)
    running = model.image_model_feat.bn1.running_mean.detach().numpy().copy()
    arrays["g3_bn1_running_mean"] = running
    arrays["g3_bn1_running_var"] = model.image_model_feat.bn1.running_var.detach().numpy().copy()

    # ---------------- G5: reference train_multimodal_model, one epoch ----------------
    torch.manual_seed(SEED_MODEL)
    models = mu.define_models(torch.device("cpu"), 7, prior)
    model = models["multimodal_model"]
    bayes_ref.set_eps_source(eps_generator_source(SEED_EPS + 1))
    opt = torch.optim.Adam(model.parameters(), lr=5e-5)
    crit = torch.nn.CrossEntropyLoss()
    loader = ListLoader(batches, batch_size=2)
    csv5 = os.path.join(tmp, "run", "multimodal_training.csv")
    os.makedirs(os.path.dirname(csv5), exist_ok=True)
    loss, acc = mm.train_multimodal_model(model, loader, crit, opt, epoch=0,
                                          device=torch.device("cpu"), model_type="multimodal",
                                          total_num_epochs=2, num_mc=2,
                                          sum_writer=SummaryWriter(), csv_path=csv5)
    out["g5_loss"], out["g5_acc"] = float(loss), float(acc)
    out["g5_csv"] = list(csv.reader(open(csv5)))
    out["g5_param_digest"] = param_digest(model)
    arrays["g5_fc2_mu_weight"] = model.fc2.mu_weight.detach().numpy().copy()
    arrays["g5_conv1_mu_kernel_img"] = model.image_model_feat.conv1.mu_kernel.detach()[:4].numpy().copy()

    # ---------------- G6: evaluate + predict (reference code) ----------------
    bayes_ref.set_eps_source(eps_generator_source(SEED_EPS + 2))
    csv6 = os.path.join(tmp, "run", "multimodal_test.csv")
    acc6 = mm.evaluate_multimodal_model(model, loader, torch.device("cpu"), epoch=0,
                                        total_num_epochs=2, num_mc=3, model_type="multimodal",
                                        csv_path=csv6)
    out["g6_eval_acc"] = float(acc6)
    out["g6_eval_csv"] = list(csv.reader(open(csv6)))
    bayes_ref.set_eps_source(eps_generator_source(SEED_EPS + 3))
    pred_loader = [(b["main_image"], b["bathy_image"], b["sss_image"], [f"img{i}_{j}" for j in range(2)])
                   for i, b in enumerate(batches)]
    csv6p = os.path.join(tmp, "pred.csv")
    # predictors.py:55 autocasts to bf16 on CPU and then crashes at :74 (`.numpy()` of a
    # bf16 tensor is unsupported) — the reference's CPU predict path cannot run as-is.
    # The golden is taken with autocast disabled (fp32), i.e. the reference maths at fp32.
    real_autocast = torch.amp.autocast
    torch.amp.autocast = lambda *a, **k: real_autocast(device_type="cpu", enabled=False)
    try:
        pr.multimodal_predict_and_save(model, pred_loader, torch.device("cpu"), csv6p,
                                       num_mc_samples=4)
    finally:
        torch.amp.autocast = real_autocast
    out["g6_predict_csv"] = list(csv.reader(open(csv6p)))

    # ---------------- G7: reference train_unimodal_model (config-1 path) ----------------
    torch.manual_seed(SEED_MODEL)
    models = mu.define_models(torch.device("cpu"), 7, prior)
    uni = models["image_model"]
    bayes_ref.set_eps_source(eps_generator_source(SEED_EPS + 4))
    opt = torch.optim.Adam(uni.parameters(), lr=1e-5)
    csv7 = os.path.join(tmp, "run", "image.csv")
    acc7, loss7 = um.train_unimodal_model(uni, loader, crit, opt, epoch=1, total_num_epochs=3,
                                          num_mc=2, sum_writer=SummaryWriter(),
                                          device=torch.device("cpu"), model_type="image",
                                          csv_path=csv7)
    out["g7_acc"], out["g7_loss"] = float(acc7), float(loss7)
    out["g7_csv"] = list(csv.reader(open(csv7)))
    out["g7_param_digest"] = param_digest(uni)
    bayes_ref.set_eps_source(None)

    with open(os.path.join(here, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    np.savez_compressed(os.path.join(here, "golden.npz"), **arrays)
    print(json.dumps({k: v for k, v in out.items() if not k.endswith("csv")}, indent=1)[:2000])


def loops_golden(mu, SummaryWriter, prior, tmp, here):
    """G8: train/loop_utils.py:162-250 train_and_evaluate_multimodal_model (2 epochs, one
    train and one test batch, num_mc=2; StepLR(step_size=1, gamma=0.5) so the scheduler's
    two steps per epoch (:233, :246) show in the CSV lr column), optimizer and scheduler from
    the reference's define_optimizers_and_schedulers (:13-63).
    G9: train_and_evaluate_unimodal_model (:65-159; epochs range(1, 3)) on the image model."""
    lu = importlib.import_module("Multimodal_AUV.train.loop_utils")
    batches = make_batches(SEED_DATA, n_batches=2, B=2, S_opt=64, S_son=64)
    out = {}
    opt_p = {k: {"lr": 5e-5} for k in ("image_model", "bathy_model", "sss_model",
                                        "multimodal_model")}
    sch_p = {k: {"step_size": 1, "gamma": 0.5} for k in opt_p}
    torch.manual_seed(SEED_MODEL)
    models = mu.define_models(torch.device("cpu"), 7, prior)
    crit, opts, schs = lu.define_optimizers_and_schedulers(models, opt_p, sch_p)
    bayes_ref.set_eps_source(eps_generator_source(SEED_EPS + 5))
    d8 = os.path.join(tmp, "g8", "csvs")
    lu.train_and_evaluate_multimodal_model(
        ListLoader(batches[:1], 2), ListLoader(batches[1:], 2), models["multimodal_model"], crit,
        opts["multimodal_model"], schs["multimodal_model"], num_epochs=2, num_mc=2,
        device=torch.device("cpu"), model_type="multimodal", bathy_patch_type=None,
        sss_patch_type=None, csv_path=d8, sum_writer=SummaryWriter())
    out["g8_train_csv"] = list(csv.reader(open(os.path.join(d8, "multimodal_training.csv"))))
    out["g8_test_csv"] = list(csv.reader(open(os.path.join(d8, "multimodal_test.csv"))))
    out["g8_lr_after"] = opts["multimodal_model"].param_groups[0]["lr"]
    out["g8_param_digest"] = param_digest(models["multimodal_model"])
    bayes_ref.set_eps_source(eps_generator_source(SEED_EPS + 6))
    d9 = os.path.join(tmp, "g9")
    os.makedirs(d9, exist_ok=True)
    lu.train_and_evaluate_unimodal_model(
        models["image_model"], ListLoader(batches[:1], 2), ListLoader(batches[1:], 2), crit,
        opts["image_model"], schs["image_model"], num_epochs=3, device=torch.device("cpu"),
        model_name="image", save_dir=d9, num_mc=2, sum_writer=SummaryWriter())
    out["g9_train_csv"] = list(csv.reader(open(os.path.join(d9, "image.csv"))))
    out["g9_eval_csv"] = list(csv.reader(open(os.path.join(d9, "image_evaluate.csv"))))
    out["g9_lr_after"] = opts["image_model"].param_groups[0]["lr"]
    out["g9_param_digest"] = param_digest(models["image_model"])
    bayes_ref.set_eps_source(None)
    with open(os.path.join(here, "golden_loops.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1)[:3000])


def staging_golden(here):
    """G10: the reference's simulate_underwater_degradation
    (Examples/"Example training with image noise.py":55-93) on seeded inputs: the function's
    own definition is taken from the script (its module imports the whole training stack and
    its file name has spaces) and run as written."""
    import ast
    path = os.path.join(REF_PKG, "Examples", "Example training with image noise.py")
    tree = ast.parse(open(path).read())
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef)
              and n.name == "simulate_underwater_degradation")
    ns = {"torch": torch}
    exec(compile(ast.Module(body=[fn], type_ignores=[]), path, "exec"), ns)
    sim = ns["simulate_underwater_degradation"]
    g = torch.Generator().manual_seed(SEED_DATA + 10)
    clean = torch.randn(2, 3, 8, 12, generator=g)            # a normalised optical batch
    ones = torch.ones(2, 1, 8, 12)
    dmap = torch.rand(2, 1, 8, 12, generator=g) * 3
    arrays = {"clean": clean.numpy(), "dmap": dmap.numpy()}
    for i, (turb, depth) in enumerate(((0.3, 1), (1.5, 1), (0.9, 2.5))):
        arrays[f"uniform_{i}"] = sim(clean, ones, turb, depth).numpy()
        arrays[f"map_{i}"] = sim(clean, dmap, turb, depth).numpy()
    np.savez_compressed(os.path.join(here, "golden_staging.npz"), **arrays)
    print("golden_staging.npz:", list(arrays))


if __name__ == "__main__":
    main()
