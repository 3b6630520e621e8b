"""The bench harness the driver's 8-GPU run executes, rehearsed with two and four ranks on one
MI355X (torch.distributed.run, gloo over CUDA tensors; RCCL needs one GPU per rank):
DistributedMC training with the MAX-over-ranks timing, the configs[4] training legs, and the
MC-sharded predictor legs — at a small batch so each runs in about a minute; four ranks with
10 MC samples shard unevenly (3, 3, 2, 2), and the sharded statistics equal one rank's."""
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


def test_bench_world4_gloo_uneven_mc_shards():
    """four ranks on one GPU, 10 MC samples over 4 ranks (3, 3, 2, 2)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "4", "--backend", "gloo",
           "--steps", "2", "--warmup", "1", "--batch", "2", "--num-mc", "2",
           "--optical", "64", "--sonar", "64", "--infer-batch", "4", "--infer-mc", "10",
           "--no-sweep", "--no-infer-sweep", "--no-infer-fp32", "--exact-steps", "0",
           "--bf16-steps", "1", "--no-roofline", "--no-cpu-baseline"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["config"]["global_batch"] == 8
    assert d["config"]["parallelism"] == "dp4" and d["value"] > 0
    assert d["inference"]["sharding"] == "mc" and d["inference"]["num_mc"] == 10
    assert d["inference"]["value"] > 0 and d["bf16_train"]["value"] > 0
    c = d["comm"]
    assert c is not None and c["buckets_per_step"] >= 1 and c["exposed_allreduce_ms_per_step"] > 0
    assert 0 < c["step_ms_per_rank_min"] <= c["step_ms_per_rank_max"] == d["ms_per_step"]


def test_mc_sharded_statistics_equal_single_rank(tmp_path):
    """The MC-sharded predictor (predict.mc_statistics with a process group: 10 samples over 4
    ranks, 3 / 3 / 2 / 2, in chunks of 2) against one rank on the same model, seed and batch:
    the ranks draw disjoint sample ranges of the rank-0 Philox stream, so every sample's logits
    are the single-rank ones and only the float64 sum order of the all-reduced sufficient
    statistics differs — f16 (autocast) and fp32."""
    worker = os.path.join(ROOT, "tests", "ranks_predict_worker.py")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    out4, out1 = str(tmp_path / "w4.json"), str(tmp_path / "w1.json")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "4", "--master-addr", "127.0.0.1", "--master-port",
                        str(_free_port()), worker, out4], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    env1 = {k: v for k, v in env.items()
            if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, worker, out1], cwd=ROOT, env=env1, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    a, b = json.load(open(out4)), json.load(open(out1))
    assert a["world"] == 4 and b["world"] == 1
    import numpy as np
    for prec in ("f16", "fp32"):
        assert a[prec]["pred"] == b[prec]["pred"], prec
        for k in ("var", "aleatoric", "predictive_entropy", "mean_prob"):
            x, y = np.array(a[prec][k]), np.array(b[prec][k])
            err = np.abs(x - y).max()
            print(f"{prec} {k}: max |4 ranks - 1 rank| {err:.3e} (|ref| <= {np.abs(y).max():.3e})")
            assert err <= 1e-6 * max(1.0, np.abs(y).max()), (prec, k, err)
