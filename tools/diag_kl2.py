"""How many KL backward calls does one drop-in unimodal training step make?"""
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
import Multimodal_AUV.train.unimodal as um  # noqa: E402
from Multimodal_AUV.models.model_utils import define_models  # noqa: E402

DEV = torch.device("cuda")
b = make_batches(SEED_DATA, 2, B=2, S_opt=64, S_son=64)
name = "model.layer4.2.conv2.rho_kernel"
for variant in ("fused_adam", "train_then_eval", "driver"):
    torch.manual_seed(SEED_MODEL)
    o = oracle_define(None, 7, DEFAULT_PRIOR)["image_model"]
    torch.manual_seed(SEED_MODEL)
    m = define_models(DEV, 7, DEFAULT_PRIOR)["image_model"]
    m.load_state_dict(o.state_dict())
    m = m.to(DEV)
    root_state(m).eps_provider = ReplayEps(m, forward_order(copy.deepcopy(o), b[0]["main_image"]),
                                           SEED_EPS + 6)
    from mauv.optim import FusedAdam
    opt = FusedAdam(m.parameters(), lr=5e-5)
    with tempfile.TemporaryDirectory() as d:
        if variant == "driver":
            import Multimodal_AUV.train.loop_utils as lu
            lu.train_and_evaluate_unimodal_model(m, ListLoader(b[:1], 2), ListLoader(b[1:], 2),
                                                 torch.nn.CrossEntropyLoss(), opt,
                                                 torch.optim.lr_scheduler.StepLR(opt, 1, 0.5),
                                                 num_epochs=2, device=DEV, model_name="image",
                                                 save_dir=d, num_mc=2, sum_writer=NullWriter())
        else:
            um.train_unimodal_model(m, ListLoader(b[:1], 2), torch.nn.CrossEntropyLoss(), opt,
                                    epoch=1, total_num_epochs=3, num_mc=2,
                                    sum_writer=NullWriter(), device=DEV, model_type="image",
                                    csv_path=os.path.join(d, "x.csv"))
        if variant == "train_then_eval":
            g0 = dict(m.named_parameters())[name].grad.clone()
            um.evaluate_unimodal_model(m, ListLoader(b[1:], 2), DEV, 1, os.path.join(d, "e.csv"),
                                       3, 2, "image")
            print("eval changed grad:", (dict(m.named_parameters())[name].grad - g0).abs().max().item())
    oo = copy.deepcopy(o)
    oopt = torch.optim.SGD(oo.parameters(), lr=0.0)
    bayes_ref.set_eps_source(eps_generator_source(SEED_EPS + 6))
    try:
        loops_ref.train_step_unimodal(oo, b[0]["main_image"], b[0]["label"],
                                      torch.nn.CrossEntropyLoss(), oopt, 1, 3, 2, 2)
    finally:
        bayes_ref.set_eps_source(None)
    g = dict(m.named_parameters())[name].grad.double().cpu().reshape(-1)
    gt = dict(oo.named_parameters())[name].grad.double().reshape(-1)
    print(variant, "kl_bwd_count", root_state(m).kl_bwd_count, "median(g_hip - g_oracle)",
          (g - gt).median().item())
