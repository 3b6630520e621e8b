"""utils/device.py surface (device.py:6-81): single device, the reference's DataParallel for
foreign modules (as unittests/test_utils.py:56-73 assert), and an actionable error — not a
silent single-GPU fallback — for a mauv model spread over several devices in one process."""
from unittest import mock

import pytest
import torch
import torch.nn as nn


def test_single_device_and_foreign_dataparallel(monkeypatch):
    from Multimodal_AUV.utils.device import move_model_to_device, move_models_to_device
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    net = nn.Linear(3, 2)
    assert move_model_to_device(net, torch.device("cpu")) is net
    with mock.patch("torch.nn.DataParallel") as dp, mock.patch.object(nn.Linear, "to",
                                                                      lambda self, d: self):
        move_model_to_device(nn.Linear(3, 2), torch.device("cpu"), device_ids=[0, 1])
        dp.assert_called_once()
        assert dp.call_args.kwargs["device_ids"] == [0, 1]
    d = move_models_to_device({"image_model": nn.Linear(2, 2), "multimodal_model": None},
                              [torch.device("cpu")])
    assert isinstance(d["image_model"], nn.Linear) and d["multimodal_model"] is None


def test_mauv_model_multi_device_single_process_raises(monkeypatch):
    from Multimodal_AUV.utils.device import move_models_to_device
    from bayesian_torch.layers import LinearReparameterization
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    models = {"multimodal_model": nn.Sequential(LinearReparameterization(3, 2))}
    devs = [torch.device("cuda", 0), torch.device("cuda", 1)]
    with pytest.raises(RuntimeError, match="torchrun --nproc-per-node 2"):
        move_models_to_device(models, devs, use_multigpu_for_multimodal=True)


def test_bench_refuses_gpus_unequal_world_size():
    """Under a launcher, --gpus must equal WORLD_SIZE: bench.py exits non-zero before it
    imports the model or touches a GPU."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr, (r.returncode, r.stderr[-500:])
