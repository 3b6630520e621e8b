"""The bench harness the driver's 8-GPU run executes, rehearsed with two ranks on one MI355X
(torch.distributed.run, gloo over CUDA tensors; RCCL needs one GPU per rank): DistributedMC
training with the MAX-over-ranks timing, the configs[4] training legs, and the MC-sharded
predictor legs — at a small batch so it runs in about a minute."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_world2_gloo_one_gpu():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
           "--steps", "2", "--warmup", "1", "--batch", "4", "--num-mc", "2",
           "--optical", "64", "--sonar", "64", "--sweep-batch", "2", "--leg-steps", "1",
           "--infer-batch", "8", "--infer-mc", "6", "--infer-sweep-batch", "4",
           "--infer-sweep-mc", "4", "--exact-steps", "0", "--bf16-steps", "1",
           "--no-roofline", "--no-cpu-baseline"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]          # rank 0 prints the one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 8
    assert d["config"]["parallelism"] == "dp2" and d["value"] > 0
    assert d["bf16_train"]["value"] > 0
    assert d["inference"]["sharding"] == "mc" and d["inference"]["value"] > 0
    c = d["comm"]                                      # the multi-rank line explains itself
    assert c["exchange_dtype"] == "fp32" and c["buckets_per_step"] >= 1
    assert c["grad_bytes_per_step"] == 4 * c["arena_values"]
    assert c["overlapped_trunk_slices_per_step"] >= 1
    assert c["exposed_allreduce_ms_per_step"] > 0
    assert 0 < c["step_ms_per_rank_min"] <= c["step_ms_per_rank_max"] == d["ms_per_step"]
    for leg in ("sonar128", "sonar512", "num_mc12", "sonar128_bf16", "sonar512_bf16"):
        assert d["train_sweep"][leg]["value"] > 0, d["train_sweep"]
    for leg in ("sonar128", "sonar512", "main_py_b8_mc12"):
        assert d["infer_sweep"][leg]["sharding"] == "mc" and d["infer_sweep"][leg]["value"] > 0


def test_bench_gpus2_without_torchrun_starts_two_ranks():
    """`python bench.py --gpus 2` with no launcher starts its own two ranks (VERDICT r4
    missing 1: --gpus was parsed and ignored, so the driver's form of the command would have
    measured one GPU)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
           "--steps", "2", "--warmup", "1", "--batch", "2", "--num-mc", "2",
           "--optical", "64", "--sonar", "64", "--no-infer", "--no-sweep", "--no-bf16",
           "--exact-steps", "0", "--no-roofline", "--no-cpu-baseline"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["comm"] is not None and d["comm"]["buckets_per_step"] >= 1
