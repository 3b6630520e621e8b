"""Rank-aware drop-in loops under DistributedMC (torchrun, one process per GPU), on CPU with
gloo (world 2): only rank 0 writes CSV rows / checkpoints, the epoch figures cover every
rank's batches, and the loops move batches to the MODEL's device — the reference scripts keep
passing ``devices[0]`` (Example_training_from_scratch.py:93) while under torchrun each rank's
model sits on cuda:LOCAL_RANK (mauv.device.move_model_to_device)."""
import csv
import os

import pytest
import torch
import torch.multiprocessing as mp
import torch.nn as nn

from tests.test_ddp_cpu import _free_port, _init
from tests.test_dropin_cpu import TinyTriModal, _batches
from tests.helpers import ListLoader, NullWriter

KL = 0.05


def _paths():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "multimodal-auv_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _loop_worker(rank, world, port, q):
    _paths()
    _init(rank, world, port)
    import Multimodal_AUV.train.multimodal as mm
    from mauv.ddp import DistributedMC
    mm.get_kl_loss = lambda model: torch.tensor(KL)
    torch.manual_seed(0)
    model = DistributedMC(TinyTriModal())
    opt = torch.optim.SGD(model.parameters(), lr=0.0)   # lr 0: both epochs see the same model
    batches = _batches(2, seed=10 + rank)                # each rank its own shard of the data
    loss, acc = mm.train_multimodal_model(model, ListLoader(batches, 4), nn.CrossEntropyLoss(),
                                          opt, epoch=1, device=torch.device("cpu"),
                                          model_type="multimodal", total_num_epochs=3, num_mc=2,
                                          sum_writer=NullWriter(),
                                          csv_path=os.path.join(q, "train.csv"))
    tacc = mm.evaluate_multimodal_model(model, ListLoader(batches, 4), torch.device("cpu"),
                                        epoch=0, total_num_epochs=2, num_mc=2,
                                        model_type="multimodal",
                                        csv_path=os.path.join(q, "test.csv"))
    # what this rank alone would count (the same model on its own batches)
    with torch.no_grad():
        outs = [model.module(b["main_image"], b["bathy_image"], b["sss_image"]) for b in batches]
    correct = sum(int((o.argmax(1) == b["label"]).sum()) for o, b in zip(outs, batches))
    torch.save((loss, acc, tacc, correct), os.path.join(q, f"r{rank}.pt"))
    import torch.distributed as dist
    dist.destroy_process_group()


def test_rank0_writes_and_epoch_figures_cover_all_ranks(tmp_path):
    mp.spawn(_loop_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (torch.load(tmp_path / f"r{r}.pt", weights_only=False) for r in range(2))
    assert r0[:3] == r1[:3]                       # every rank returns the global figures
    assert r0[1] == (r0[3] + r1[3]) / 16          # training accuracy over both ranks' 16 items
    assert r0[2] == (r0[3] + r1[3]) / 16          # evaluation accuracy likewise
    for name in ("train.csv", "test.csv"):
        rows = list(csv.reader(open(tmp_path / name)))
        assert len(rows) == 2, rows               # header + ONE row (rank 0), not one per rank
    assert float(list(csv.reader(open(tmp_path / "test.csv")))[1][3]) == r0[2]


class _FakeParam:
    is_cuda = True
    device = torch.device("cuda", 1)


class _RankModel(nn.Module):
    """Stands for a mauv model that torchrun placed on cuda:1 (no GPU here)."""

    def mc_forward(self, *a):
        raise AssertionError

    def parameters(self, recurse=True):
        return iter([_FakeParam()])


def test_batches_follow_the_model_device():
    _paths()
    from mauv.train import loop_device
    assert loop_device(_RankModel(), torch.device("cuda", 0)) == torch.device("cuda", 1)
    assert torch.device(loop_device(_RankModel(), "cuda:1")) == torch.device("cuda", 1)
    host = TinyTriModal()   # foreign model: the caller's device is kept
    assert loop_device(host, torch.device("cpu")) == torch.device("cpu")


def test_kernel_operand_on_another_device_is_refused(monkeypatch):
    """ops refuses a tensor that is not on the device whose stream the launch would use."""
    _paths()
    from mauv import ops

    class T:
        is_cuda = True
        dtype = torch.float32
        device = torch.device("cuda", 1)
        shape = (4,)

        def is_contiguous(self):
            return True
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)
    with pytest.raises(ValueError, match="cuda:0"):
        ops._f32(T())
