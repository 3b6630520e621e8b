"""Unimodal ResNet50Custom at 16-bit: the HIP path's deviation from the fp32 oracle next to
torch's own autocast run of the same oracle model on the GPU (same weights, same epsilons)."""
import copy
import os
import sys

import torch

R = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "multimodal-auv_amd"))
from oracle import model_ref, bayes_ref  # noqa: E402
from oracle.bayes_ref import dnn_to_bnn as o_dnn_to_bnn  # noqa: E402
from mauv.models import ResNet50Custom  # noqa: E402
from mauv.layers import dnn_to_bnn  # noqa: E402
from mauv.engine import root_state, set_precision  # noqa: E402
from tests.helpers import DEFAULT_PRIOR, EpsBridge  # noqa: E402


class Replay:
    def __init__(self, log):
        self.log, self.i = log, 0

    def __call__(self, layer, name, shape):
        e = self.log[self.i][2]
        self.i += 1
        assert tuple(e.shape) == tuple(shape)
        return e


for cin, S, B in ((3, 64, 2), (3, 160, 4), (2, 160, 4)):
    torch.manual_seed(3)
    o = model_ref.ResNet50Custom(cin, 7)
    o_dnn_to_bnn(o, DEFAULT_PRIOR)
    og = copy.deepcopy(o).cuda()
    m = ResNet50Custom(cin, 7)
    dnn_to_bnn(m, DEFAULT_PRIOR)
    m.load_state_dict(o.state_dict())
    m = m.cuda()
    torch.manual_seed(4)
    x = torch.randn(B, cin, S, S)
    bridge = EpsBridge(o, m, 17)
    with bridge, torch.no_grad():
        ol = torch.stack([o(x) for _ in range(2)])
    log = list(bridge.src.log)
    bridge.collect()
    for dt in (torch.bfloat16, torch.float16):
        bayes_ref.set_eps_source(Replay(log))
        try:
            with torch.no_grad(), torch.autocast("cuda", dtype=dt):
                tl = torch.stack([og(x.cuda()) for _ in range(2)]).float().cpu()
        finally:
            bayes_ref.set_eps_source(None)
        root_state(m).eps_provider = bridge.provider
        root_state(m).offset = 0
        set_precision(m, dt)
        with torch.no_grad():
            lg = m.mc_forward(x.cuda(), 2)
        print(cin, S, B, dt, "hip max|d|", round((lg.double().cpu() - ol.double()).abs().max().item(), 4),
              "torch-autocast max|d|", round((tl.double() - ol.double()).abs().max().item(), 4),
              "max|ref|", round(ol.abs().max().item(), 3))
