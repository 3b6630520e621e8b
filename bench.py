#!/usr/bin/env python3
"""Benchmark: tri-modal Bayesian MC training step (BASELINE.json configs[1]) on MI355X.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (driver, one rank per GPU, RCCL)

A step = one reference training batch (train/multimodal.py:104-146) of synthetic triplets
already resident in HBM: num_mc=5 stochastic forwards (one batched launch per layer), KL,
cross-entropy, backward, RCCL gradient all-reduce (N>1), NaN/Inf guard, Adam step.
Workload per GPU: B=64 triplets, optical 3x224x224 ~N(0,1), bathy 3x256x256 ~U[0,1) with
channel 2 = 0, SSS 1x256x256 ~U[0,1), 7 classes, fp32 (weak scaling: 64 per GPU).

Also reported: the same step with bf16 trunks (configs[2]'s per-GPU slice, `bf16_train`),
MC inference (configs[3]: 100 passes over 256 triplets, MC-sharded across ranks, under
torch.autocast as the reference predictor runs it -> f16 trunks), the roofline of the dominant
kernel family (implicit-GEMM conv fwd/dgrad/wgrad, HIP-event timed inside this run), and the
reference-semantics CPU path (oracle/, torch-CPU fp32, sequential MC loop) timed on a bounded
sample on this host.
"""
import argparse
import json
import os
import platform
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
import sys  # noqa: E402
for _p in (REPO, os.path.join(REPO, "multimodal-auv_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "triplets/sec training + MC-samples/sec inference, 7-class BNN, 1/2/4/8 MI355X"
FP32_MFMA_PEAK_TF = 157.3   # MI355X_MICROARCH.md: f32-in MFMA = vector peak (spec)
BF16_MFMA_PEAK_TF = 2500.0  # MI355X_MICROARCH.md: dense bf16/f16 MFMA (no sparsity)
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E
# fp32 GEMM arithmetic of the convs (include/mauv.h mauv_set_f32_math): "split" issues six
# bf16 MFMA plane products per fp32 product, "exact" one f32 MFMA
F32_PEAK_TF = {"split": BF16_MFMA_PEAK_TF / 6, "split1": BF16_MFMA_PEAK_TF / 6,
               "split3": BF16_MFMA_PEAK_TF / 3, "exact": FP32_MFMA_PEAK_TF}


def progress(msg):
    """One line per bench leg on rank 0's stderr (a run that prints nothing for minutes looks
    hung to the harness)."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def synthetic_batch(B, S_opt, S_son, device, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(B, 3, S_opt, S_opt, generator=g)
    bathy = torch.rand(B, 3, S_son, S_son, generator=g)
    bathy[:, 2] = 0
    sss = torch.rand(B, 1, S_son, S_son, generator=g)
    y = torch.randint(0, 7, (B,), generator=g)
    return [t.to(device) for t in (x, bathy, sss, y)]


def _host_cpu():
    """CPU model, physical cores of the host, CPUs this process may run on."""
    model, cores = platform.processor() or platform.machine(), set()
    try:
        phys = core = None
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name":
                    model = v
                elif k == "physical id":
                    phys = v
                elif k == "core id":
                    core = v
                elif not k and phys is not None:
                    cores.add((phys, core))
                    phys = core = None
    except OSError:
        pass
    try:
        aff = sorted(os.sched_getaffinity(0))
    except AttributeError:
        aff = list(range(os.cpu_count() or 1))
    # physical cores among the CPUs this process may run on (SMT siblings counted once)
    phys = set()
    for c in aff:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            with open(base + "physical_package_id") as f:
                pk = f.read().strip()
            with open(base + "core_id") as f:
                phys.add((pk, f.read().strip()))
        except OSError:
            phys.add(("?", c))
    return {"cpu_model": model, "host_physical_cores": len(cores) or None,
            "host_logical_cpus": os.cpu_count(), "usable_cpus": len(aff),
            "usable_physical_cores": len(phys),
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(args):
    """Reference-semantics CPU path (oracle = torch-CPU restatement of the reference's loops:
    sequential MC loop, per-pass epsilon draws and KL, torch Adam) timed on bounded samples
    of the same workloads on this host:
      * configs[1] training (the headline unit): B=2, num_mc=2 at full resolution, scaled to
        num_mc=5 (work is linear in num_mc and B);
      * configs[0] in full: unimodal optical BNN (ResNet50Custom(3, 7)), B=8, 224 px,
        num_mc=5, train/unimodal.py's step;
      * configs[3] inference: predictors.py's MC loop at B=4, num_mc=2 (fp32: the reference's
        CPU autocast crashes at predictors.py:74), per MC-sample triplet."""
    from oracle.model_ref import define_models, DEFAULT_PRIOR
    from oracle import loops_ref
    host = _host_cpu()
    prev_threads = torch.get_num_threads()
    torch.manual_seed(0)
    models = define_models(None, 7, DEFAULT_PRIOR)
    model = models["multimodal_model"]
    # torch.set_num_threads(<physical cores>).  On a shared GPU box every
    # physical core is not this job's (OMP_NUM_THREADS is the box's per-GPU share), and
    # oversubscribed threads run the oracle ~13x slower (round 3: 0.042 triplets/s at 128
    # threads vs 0.56 at 16) — so the thread count is CALIBRATED: one trunk forward timed at
    # the box's share, 2x, 4x and the physical cores of the affinity set; the fastest is used
    # and every candidate is reported.
    xc, _, _, _ = synthetic_batch(2, args.optical, args.sonar, "cpu", 5)
    cands = sorted({max(1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)) * k
                    for k in (1, 2, 4)} | {max(1, host["usable_physical_cores"])})
    calib = {}
    with torch.no_grad():
        for n in cands:
            torch.set_num_threads(n)
            model.image_model_feat(xc)                   # warm-up at this thread count
            t0 = time.perf_counter()
            model.image_model_feat(xc)
            calib[n] = round(time.perf_counter() - t0, 4)
    threads = min(calib, key=calib.get)
    torch.set_num_threads(threads)
    opt = torch.optim.Adam(model.parameters(), lr=5e-5)
    crit = torch.nn.CrossEntropyLoss()
    Bc, Nc = 2, 2
    x, b, s, y = synthetic_batch(Bc, args.optical, args.sonar, "cpu", 1)
    loops_ref.train_step_multimodal(model, x, b, s, y, crit, opt, 0, 2, Nc, Bc)  # warm-up
    t0 = time.perf_counter()
    reps = 2
    for _ in range(reps):
        loops_ref.train_step_multimodal(model, x, b, s, y, crit, opt, 0, 2, Nc, Bc)
    dt = (time.perf_counter() - t0) / reps
    per_triplet = dt / Bc * (args.num_mc / Nc)
    out = {"value": round(1.0 / per_triplet, 4), "unit": "triplets/s", "cores": threads,
           "kind": "port",
           "sample": f"oracle train step, B={Bc}, num_mc={Nc} (scaled x{args.num_mc}/{Nc} to "
                     f"num_mc={args.num_mc}), {args.optical}/{args.sonar} px, torch-CPU fp32, "
                     f"{reps} timed steps of {dt:.2f} s"}
    out.update(host)
    out["threads_calibration_s"] = {str(k): v for k, v in calib.items()}
    # configs[0]: the unimodal CPU path, timed in full
    uni = models["image_model"]
    uopt = torch.optim.Adam(uni.parameters(), lr=5e-5)
    xu, _, _, yu = synthetic_batch(8, args.optical, args.sonar, "cpu", 2)
    loops_ref.train_step_unimodal(uni, xu, yu, crit, uopt, 0, 2, args.num_mc, 8)   # warm-up
    t0 = time.perf_counter()
    for _ in range(reps):
        loops_ref.train_step_unimodal(uni, xu, yu, crit, uopt, 0, 2, args.num_mc, 8)
    du = (time.perf_counter() - t0) / reps
    out["configs0_unimodal"] = {
        "value": round(8 / du, 4), "unit": "images/s", "ms_per_step": round(du * 1e3, 1),
        "sample": f"configs[0] in full: ResNet50Custom(3,7) BNN, B=8, {args.optical} px, "
                  f"num_mc={args.num_mc}, train/unimodal.py step, {reps} timed steps"}
    # configs[3]: MC inference
    Bi, Ni = 4, 2
    xi, bi, si, _ = synthetic_batch(Bi, args.optical, args.sonar, "cpu", 3)
    loops_ref.predict_batch(model, xi, bi, si, Ni)   # warm-up
    t0 = time.perf_counter()
    for _ in range(reps):
        loops_ref.predict_batch(model, xi, bi, si, Ni)
    di = (time.perf_counter() - t0) / reps
    out["inference"] = {
        "value": round(Bi * Ni / di, 4), "unit": "MC-samples/s",
        "sample": f"predictors.py MC loop, B={Bi}, num_mc={Ni}, {args.optical}/{args.sonar} px, "
                  f"fp32, {reps} timed batches of {di:.2f} s (per MC-sample triplet; the "
                  f"GPU number is B=256, num_mc=100)"}
    torch.set_num_threads(prev_threads)
    return out


def pmc_traffic(family="fp32"):
    """HBM bytes per conv launch from the committed PMC summary of this same command
    (tools/pmc_traffic.py; separate FETCH_SIZE and WRITE_SIZE passes, FETCH_SIZE doubled per
    MI355X_MICROARCH.md's gfx950 correction).  PMC collection serialises kernels, so it runs
    as its own profiled invocation; the newest profiles/round*_conv_traffic.json (fp32 split
    convs) or round*_bf16_conv_traffic.json (the 16-bit family) is used."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "round*_conv_traffic.json")))
    files = [f for f in files if ("_bf16_" in os.path.basename(f)) == (family == "bf16")]
    if not files:
        return None, None, None
    with open(files[-1]) as f:
        d = json.load(f)
    return d, os.path.relpath(files[-1], REPO), d.get("library_sha16")


def library_sha16():
    """sha256 prefix of the libmauv_hip.so this process loaded (the PMC traffic summary records
    the library it profiled, so the line says whether the two match)."""
    import hashlib
    from mauv import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def roofline_step(step_fn, peak=FP32_MFMA_PEAK_TF, traffic="fp32", suffix="",
                  kernel="conv_gemm_f32 (implicit-GEMM fwd+dgrad+wgrad, all launches of one step)"):
    """Roofline of one step's implicit-GEMM launches of one precision (suffix "" = fp32,
    "_bfloat16" = the 16-bit trunks; the fp32 fusion-head GEMMs are then excluded).  The
    three trunks run one after another in this step (no concurrent trunk streams), so each
    launch's HIP-event duration is the kernel's own."""
    from mauv import ops, engine
    prev, engine.TRUNK_STREAMS = engine.TRUNK_STREAMS, False
    ops.PROFILE = []
    try:
        torch.cuda.synchronize()
        step_fn()
        torch.cuda.synchronize()
    finally:
        engine.TRUNK_STREAMS = prev
    rows, ops.PROFILE = ops.PROFILE, None
    by = {}
    nbytes = 0.0
    roof_ms, n_hbm = 0.0, 0
    fold = [0, 0.0, 0.0, 0.0]   # launches, flops, bytes, ms of the block-output folds
    for kind, fl, nb, nl, e0, e1 in rows:
        if (suffix and not kind.endswith(suffix)) or (not suffix and "_" in kind):
            continue
        ms = e0.elapsed_time(e1)
        if kind.startswith("fold_"):
            # conv1 launches that also form the previous block's output: an
            # HBM-bound pass fused into a GEMM, reported beside the MFMA roofline, not in it
            fold[0] += nl
            fold[1] += fl
            fold[2] += nb
            fold[3] += ms
            continue
        # this launch's own roofline time: its FLOPs at the MFMA peak or its algorithmic bytes
        # at the HBM peak, whichever is longer
        t_fl, t_hbm = fl / (peak * 1e12) * 1e3, nb / (HBM_PEAK_GBS * 1e9) * 1e3
        roof_ms += max(t_fl, t_hbm)
        n_hbm += nl if t_hbm > t_fl else 0
        d = by.setdefault(kind, [0, 0.0, 0.0])
        d[0] += nl
        d[1] += fl
        d[2] += ms
        nbytes += nb
    tot_fl = sum(v[1] for v in by.values())
    tot_ms = sum(v[2] for v in by.values())
    n = sum(v[0] for v in by.values())
    achieved = tot_fl / (tot_ms * 1e-3) / 1e12
    pmc, tsrc, tsha = pmc_traffic(traffic) if traffic else (None, None, None)
    traffic = pmc["bytes_per_launch"] if pmc else None
    pmc_launches = pmc.get("launches") if pmc else None
    pfold = (pmc or {}).get("per_family", {}).get("conv_fold16")
    lsha = library_sha16()
    alg = nbytes / max(n, 1)
    return {
        "bound": "mfma", "achieved": round(achieved, 2), "peak": peak,
        "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic,
        "traffic_unit": "HBM bytes per launch (2*FETCH_SIZE + WRITE_SIZE, rocprofv3 PMC)",
        "traffic_source": tsrc, "traffic_library_sha16": tsha, "library_sha16": lsha,
        "traffic_matches_library": tsha == lsha,
        "algorithmic_bytes_per_launch": round(alg),
        # the PMC summary covers the same launch set as `launches` (the fold family apart): the
        # ratio is then HBM bytes moved per algorithmic byte of this family
        "traffic_launches": pmc_launches,
        "traffic_ratio": round(traffic / alg, 3) if traffic and alg else None,
        "kernel": kernel,
        "launches": n, "avg_launch_us": round(tot_ms * 1e3 / max(n, 1), 2),
        "algorithmic_gflop_per_launch": round(tot_fl / max(n, 1) / 1e9, 3),
        "conv_ms_per_step": round(tot_ms, 2),
        "per_launch_roofline": {
            "ms": round(roof_ms, 2), "frac": round(roof_ms / tot_ms, 4),
            "hbm_bound_launches": n_hbm,
            "note": "sum over launches of max(FLOPs / MFMA peak, algorithmic bytes / HBM peak) "
                    "against the summed measured durations"},
        "breakdown": {k: {"launches": v[0], "gflop": round(v[1] / 1e9, 1),
                          "ms": round(v[2], 2), "tflops": round(v[1] / (v[2] * 1e-3) / 1e12, 1)}
                      for k, v in by.items()},
        "fold": None if not fold[0] else {
            "launches": fold[0], "gflop": round(fold[1] / 1e9, 1), "ms": round(fold[3], 2),
            "algorithmic_gbytes": round(fold[2] / 1e9, 2),
            "tbytes_per_s": round(fold[2] / (fold[3] * 1e-3) / 1e12, 2),
            "algorithmic_bytes_per_launch": round(fold[2] / fold[0]),
            "traffic": round(pfold["bytes_per_launch"]) if pfold else None,
            "traffic_launches": pfold["launches"] if pfold else None,
            "traffic_ratio": round(pfold["bytes_per_launch"] / (fold[2] / fold[0]), 3)
            if pfold else None,
            "note": "conv1 launches that also form the previous block output (bn3 + residual "
                    "+ ReLU, DESIGN.md 2.20); not in achieved / frac / launches above"},
    }


def spawn_ranks(n):
    """`python bench.py --gpus N` without torchrun: N child processes of this script, rank r on
    GPU r (torch.distributed env rendezvous on 127.0.0.1), started before this parent
    initialises the GPU (it never does).  Rank 0 prints the JSON line; the exit status is the
    first failing rank's (the others are then stopped)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   GROUP_RANK="0")
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:     # a rank died: the others would wait on it forever
                    q.terminate()
        if live:
            time.sleep(0.5)
    for p in procs:
        p.wait()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node, one rank each (default: WORLD_SIZE, else 1).  "
                         "Without torchrun, N > 1 starts N rank processes itself")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64, help="triplets per GPU")
    ap.add_argument("--num-mc", type=int, default=5)
    ap.add_argument("--optical", type=int, default=224)
    ap.add_argument("--sonar", type=int, default=256)
    ap.add_argument("--infer-batch", type=int, default=256)
    ap.add_argument("--infer-mc", type=int, default=100)
    ap.add_argument("--infer-batches", type=int, default=3,
                    help="distinct batches each inference leg times (main.py's shape: 32)")
    ap.add_argument("--no-infer", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="trunk precision of the headline measurement (default fp32 = "
                         "configs[1]); bf16 = configs[2]'s per-GPU slice (profiling)")
    ap.add_argument("--no-bf16", action="store_true",
                    help="skip the bf16 training measurement (configs[2] per-GPU slice)")
    ap.add_argument("--bf16-steps", type=int, default=5)
    ap.add_argument("--no-infer-fp32", action="store_true",
                    help="skip MC inference with fp32 trunks (autocast off)")
    ap.add_argument("--no-sweep", action="store_true",
                    help="skip the per-GPU slices of configs[4] (S=128/512, B=32) and the "
                         "num_mc=12 step of main.py:310")
    ap.add_argument("--exact-steps", type=int, default=5,
                    help="also time the fp32 step with exact f32 MFMA products (0 = skip)")
    ap.add_argument("--leg-steps", type=int, default=5,
                    help="timed steps of each train_sweep leg")
    ap.add_argument("--no-infer-sweep", action="store_true",
                    help="skip configs[4]'s MC-inference legs (sonar 128 / 512 px, B=256, "
                         "N=100) and main.py's predictor call shape (B=8, num_mc=12)")
    ap.add_argument("--sweep-batch", type=int, default=32,
                    help="triplets per GPU of the configs[4] training legs (256 over 8 GPUs)")
    ap.add_argument("--infer-sweep-batch", type=int, default=256)
    ap.add_argument("--infer-sweep-mc", type=int, default=100)
    ap.add_argument("--grad-exchange", default="fp32", choices=["fp32", "bf16"],
                    help="world > 1: gradient all-reduce in fp32 (587 MB per step) or as a bf16 "
                         "copy of the arena (294 MB, mauv.ddp.DistributedMC grad_dtype)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for world > 1 (nccl = RCCL over xGMI; gloo "
                         "rehearses the multi-rank harness, e.g. two ranks on one GPU)")
    args = ap.parse_args()

    # --gpus N is honoured or refused, never silently measured on one GPU: without a launcher
    # (WORLD_SIZE unset) N > 1 ranks are started here, before this process touches the GPU;
    # under torchrun the world size must equal N
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        sys.exit(spawn_ranks(args.gpus))
    if env_world is not None and args.gpus is not None and int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world} (one rank per GPU)",
              file=sys.stderr, flush=True)
        sys.exit(2)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; a rehearsal with more ranks than GPUs (gloo) shares them round-robin
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    from mauv.models import define_models, DEFAULT_PRIOR
    from mauv.train import mc_train_step
    from mauv.predict import mc_statistics, mc_chunk
    from mauv.engine import root_state

    torch.manual_seed(0)
    model = define_models(None, 7, DEFAULT_PRIOR)["multimodal_model"].to(dev)
    if world > 1:
        from mauv.ddp import DistributedMC
        model = DistributedMC(model, grad_dtype=torch.bfloat16 if args.grad_exchange == "bf16"
                              else torch.float32)
    from mauv.optim import FusedAdam   # what mauv.loop_utils builds for GPU models
    opt = FusedAdam(model.parameters(), lr=5e-5)
    crit = torch.nn.CrossEntropyLoss()
    x, b, s, y = synthetic_batch(args.batch, args.optical, args.sonar, dev, 1234 + rank)
    if args.dtype == "bf16":
        from mauv.engine import set_precision
        set_precision(model.module if world > 1 else model, torch.bfloat16)
    kl_w = 2.0 ** 1 / 2.0 ** 30   # epoch 0 of 30 (main.py:293)

    def step():
        return mc_train_step(model, (x, b, s), y, crit, opt, args.num_mc, args.batch, kl_w)

    # world > 1: the gradient exchange's caller-stream time (waits on the trunk slices issued
    # during the backward + the rest of the arena + the 1/world scale) = exposed all-reduce
    comm_events = []
    if world > 1:
        _allreduce = model.allreduce_grads

        def allreduce_timed():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _allreduce()
            e1.record()
            comm_events.append((e0, e1))
        model.allreduce_grads = allreduce_timed

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    barrier()
    torch.cuda.synchronize()
    comm_events.clear()
    c0 = (model.n_buckets, model.n_overlapped, model.elems_reduced) if world > 1 else None
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
        if rank == 0 and args.steps > 3:
            print(f"[bench] step {i + 1}/{args.steps}", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    comm = None
    if world > 1:
        per_rank = [torch.zeros(1, dtype=torch.float64, device=dev) for _ in range(world)]
        dist.all_gather(per_rank, torch.tensor([dt], dtype=torch.float64, device=dev))
        per_rank = [float(t.item()) for t in per_rank]
        dt = max(per_rank)
        nb, no, ne = (model.n_buckets - c0[0], model.n_overlapped - c0[1],
                      model.elems_reduced - c0[2])
        esz = 2 if args.grad_exchange == "bf16" else 4
        exposed = [a.elapsed_time(b) for a, b in comm_events]
        comm = {"backend": args.backend + (" (RCCL)" if args.backend == "nccl" else ""),
                "exchange_dtype": args.grad_exchange,
                "grad_bytes_per_step": int(ne * esz / args.steps),
                "arena_values": int(root_state(model.module).arena.numel),
                "buckets_per_step": round(nb / args.steps, 2),
                "bucket_bytes": int(model.bucket_elems * esz),
                "overlapped_trunk_slices_per_step": round(no / args.steps, 2),
                "exposed_allreduce_ms_per_step": round(sum(exposed) / max(len(exposed), 1), 3),
                "step_ms_per_rank_min": round(min(per_rank) / args.steps * 1e3, 2),
                "step_ms_per_rank_max": round(max(per_rank) / args.steps * 1e3, 2),
                "note": "exposed = caller-stream time of allreduce_grads (waits on the trunk "
                        "slices all-reduced during the backward, the remaining buckets, the "
                        "1/world scale), HIP events over the timed steps"}
    triplets_s = args.batch * world * args.steps / dt
    from mauv import ops
    f32_math = ops.f32_math()
    roof = None
    if not args.no_roofline and args.dtype == "fp32":
        roof = roofline_step(step, peak=round(F32_PEAK_TF[f32_math], 1),
                             kernel=f"conv_gemm_f32 [{f32_math}] (implicit-GEMM fwd+dgrad+wgrad, "
                                    "all launches of one step)")
        roof["f32_math"] = f32_math
        roof["frac_of_f32_mfma_peak"] = round(roof["achieved"] / FP32_MFMA_PEAK_TF, 4)

    def timed(fn, steps):
        barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        barrier()
        t = time.perf_counter() - t
        if world > 1:
            tt = torch.tensor([t], device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t = tt.item()
        return t

    exact = None
    progress("roofline step done")
    if args.dtype == "fp32" and args.exact_steps > 0 and f32_math != "exact":
        progress("exact-f32 leg")
        # the same step with every fp32 product on v_mfma_f32_32x32x2_f32 (reference point)
        ops.set_f32_math("exact")
        step()
        te = timed(step, args.exact_steps)
        exact = {"value": round(args.batch * world * args.exact_steps / te, 3),
                 "unit": "triplets/s", "ms_per_step": round(te / args.exact_steps * 1e3, 2),
                 "steps": args.exact_steps, "f32_math": "exact (v_mfma_f32_32x32x2_f32)"}
        ops.set_f32_math(f32_math)

    bf16 = None
    if not args.no_bf16:
        progress("bf16 leg")
        from mauv.engine import set_precision
        set_precision(model.module if world > 1 else model, torch.bfloat16)
        step()                                   # warm-up (16-bit kernels, allocator)
        tb = timed(step, args.bf16_steps)
        bf16 = {"value": round(args.batch * world * args.bf16_steps / tb, 3),
                "unit": "triplets/s", "ms_per_step": round(tb / args.bf16_steps * 1e3, 2),
                "steps": args.bf16_steps, "dtype": "bf16",
                "config": f"configs[2] per-GPU slice: B={args.batch}/GPU (global "
                          f"{args.batch * world}), bf16 trunks (fp32 accumulation, BN "
                          f"statistics, master weights, head), num_mc={args.num_mc}"}
        if not args.no_roofline:
            bf16["roofline"] = roofline_step(
                step, peak=BF16_MFMA_PEAK_TF, traffic="bf16", suffix="_bfloat16",
                kernel="16-bit convs of one step (conv_pipe16 / conv_halo16 / conv_haloc16 / "
                       "conv_big16 / conv_expand16: implicit-GEMM fwd+dgrad+wgrad, stems as "
                       "one GEMM over shared im2col rows); "
                       "the conv1 launches that also form the previous block output: 'fold'")
        set_precision(model.module if world > 1 else model,
                      torch.bfloat16 if args.dtype == "bf16" else None)

    sweep = None
    if not args.no_sweep:
        # configs[4] per-GPU slice (B=256 over 8 GPUs = 32/GPU) at the sonar sizes the
        # headline does not cover, and main.py:310's num_mc=12 at the headline shape; same
        # model, optimiser and trunk precision as the headline.  Each leg reports its peak
        # HBM; a leg that does not fit is reported, not fatal.
        # BASELINE.md row 5 states configs[4] in bf16: its two sonar legs also run with bf16
        # trunks (the headline precision's legs stay beside them)
        from mauv.engine import set_precision
        sweep = {}
        legs = [(f"sonar{S}", args.sweep_batch, S, args.num_mc, args.dtype) for S in (128, 512)]
        legs.append(("num_mc12", args.batch, args.sonar, 12, args.dtype))
        if args.dtype != "bf16":
            legs += [(f"sonar{S}_bf16", args.sweep_batch, S, args.num_mc, "bf16")
                     for S in (128, 512)]
        core = model.module if world > 1 else model
        for name, Bs, S, nmc, ldt in legs:
            progress(f"train_sweep {name}")
            set_precision(core, torch.bfloat16 if ldt == "bf16" else None)
            opt.zero_grad(set_to_none=True)
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            torch.cuda.reset_peak_memory_stats(dev)
            try:
                xs_, bs_, ss_, ys_ = synthetic_batch(Bs, args.optical, S, dev, 4321 + rank)

                def sstep():
                    return mc_train_step(model, (xs_, bs_, ss_), ys_, crit, opt, nmc, Bs, kl_w)

                sstep()
                ts = timed(sstep, args.leg_steps)
                sweep[name] = {"value": round(Bs * world * args.leg_steps / ts, 3),
                               "unit": "triplets/s",
                               "ms_per_step": round(ts / args.leg_steps * 1e3, 2),
                               "steps": args.leg_steps,
                               "batch_per_gpu": Bs, "sonar_px": S, "optical_px": args.optical,
                               "num_mc": nmc, "dtype": ldt,
                               "peak_hbm_gib": round(torch.cuda.max_memory_allocated(dev) / 2**30, 1)}
            except torch.OutOfMemoryError as e:
                sweep[name] = {"error": "out of memory", "detail": str(e)[:200]}
            finally:
                xs_ = bs_ = ss_ = ys_ = None
        set_precision(core, torch.bfloat16 if args.dtype == "bf16" else None)
        opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()

    uni = None
    if not args.no_sweep and world == 1:
        # BASELINE configs[0] (the reference's unimodal CPU config: ResNet50Custom(3, 7) BNN,
        # B=8, 224 px, num_mc=5, train/unimodal.py) on the HIP path, beside its CPU baseline
        progress("configs[0] unimodal leg")
        torch.manual_seed(0)
        um = define_models(None, 7, DEFAULT_PRIOR)["image_model"].to(dev)
        uopt = FusedAdam(um.parameters(), lr=5e-5)
        xu, _, _, yu = synthetic_batch(8, args.optical, args.sonar, dev, 2)

        def ustep():
            return mc_train_step(um, (xu,), yu, crit, uopt, args.num_mc, 8, kl_w)
        ustep()
        tu = timed(ustep, 10)
        uni = {"value": round(8 * 10 / tu, 2), "unit": "images/s",
               "ms_per_step": round(tu / 10 * 1e3, 2), "steps": 10, "batch": 8,
               "num_mc": args.num_mc, "dtype": "fp32",
               "config": "configs[0] on the HIP path: ResNet50Custom(3, 7) BNN, B=8, "
                         f"{args.optical} px, num_mc={args.num_mc}"}
        del um, uopt
        torch.cuda.synchronize()
        torch.cuda.empty_cache()

    infer = None
    if not args.no_infer:
        progress("inference leg")
        from mauv.predict import multimodal_predict_and_save
        opt.zero_grad(set_to_none=True)
        nib = max(1, args.infer_batches)
        loader = []
        for j in range(nib):
            xi, bi, si, _ = synthetic_batch(args.infer_batch, args.optical, args.sonar, dev, 99 + j)
            loader.append((xi, bi, si, [f"tile{j}_{i}" for i in range(args.infer_batch)]))
        group = dist.group.WORLD if world > 1 else None
        pred_csv = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"mauv_bench_pred_r{rank}.csv")
        hw = [(args.optical, args.optical), (args.sonar, args.sonar), (args.sonar, args.sonar)]

        def warm(dtype):
            # Training's cached blocks are released first and the warm-up runs one full MC
            # chunk per rank, so the timed batch reuses its activation blocks instead of
            # growing (or, near the HBM limit, flushing and retrying) the caching allocator.
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            return mc_chunk(model, args.infer_batch, args.infer_mc, dtype=dtype, device=dev,
                            hw=hw)

        # the drop-in predictor exactly as a user calls it (inference/predictors.py:9-97):
        # its own torch.amp.autocast (predictors.py:55 -> f16 trunks), MC samples sharded
        # across ranks under DistributedMC, fused statistics, CSV rows written
        chunk = warm(torch.float16)
        multimodal_predict_and_save(model, loader[:1], dev, pred_csv,
                                    num_mc_samples=max(world, 2) * chunk)
        di = timed(lambda: multimodal_predict_and_save(model, loader, dev, pred_csv,
                                                       num_mc_samples=args.infer_mc), 1)
        infer = {"value": round(args.infer_mc * args.infer_batch * nib / di, 2),
                 "unit": "MC-samples/s", "batch": args.infer_batch, "num_mc": args.infer_mc,
                 "batches": nib, "ms_per_batch": round(di / nib * 1e3, 1), "mc_chunk": chunk,
                 "sharding": "mc" if world > 1 else "none",
                 "path": "Multimodal_AUV.inference.predictors.multimodal_predict_and_save",
                 "dtype": "f16 trunks (the predictor's own torch.amp.autocast, predictors.py:55)"}
        if not args.no_infer_fp32:
            # fp32 trunks: the same MC statistics with autocast off
            chunk32 = warm(torch.float32)
            with torch.no_grad():
                mc_statistics(model, *loader[0][:3], max(world, 2) * chunk32, group=group)
                d32 = timed(lambda: [mc_statistics(model, *lb[:3], args.infer_mc, group=group)
                                     for lb in loader], 1)
            infer["fp32"] = {"value": round(args.infer_mc * args.infer_batch * nib / d32, 2),
                             "unit": "MC-samples/s", "batches": nib,
                             "ms_per_batch": round(d32 / nib * 1e3, 1),
                             "mc_chunk": chunk32,
                             "dtype": "fp32 trunks (split-fp32 convs), autocast off",
                             "path": "mauv.predict.mc_statistics"}

    infer_sweep = None
    if not args.no_infer and not args.no_infer_sweep:
        # configs[4]'s MC-sharded inference at the sonar sizes the headline does not cover
        # (B=256, N=100, 224 px optical; MC samples sharded over the ranks), and the reference's
        # own predictor call shape (main.py:261-271: batch_size_unimodal=8 :315, num_mc=12
        # :310) over 32 batches — both through the drop-in multimodal_predict_and_save under
        # its own f16 autocast
        infer_sweep = {}
        legs = [(f"sonar{S}", args.infer_sweep_batch, S, args.infer_sweep_mc,
                 max(1, args.infer_batches)) for S in (128, 512)]
        legs.append(("main_py_b8_mc12", 8, args.sonar, 12, 32))
        for name, Bi, S, Ni, nb in legs:
            progress(f"infer_sweep {name}")
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            torch.cuda.reset_peak_memory_stats(dev)
            try:
                batches = []
                for j in range(nb):
                    xi_, bi_, si_, _ = synthetic_batch(Bi, args.optical, S, dev, 500 + j)
                    batches.append((xi_, bi_, si_, [f"t{j}_{i}" for i in range(Bi)]))
                pcsv = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"mauv_bench_{name}_r{rank}.csv")
                # warm-up: one MC chunk per rank (allocator blocks of the timed batch)
                ck = mc_chunk(model, Bi, Ni, dtype=torch.float16, device=dev,
                              hw=[(args.optical, args.optical), (S, S), (S, S)])
                multimodal_predict_and_save(model, batches[:1], dev, pcsv,
                                            num_mc_samples=min(Ni, max(world, 2) * ck))
                d = timed(lambda: multimodal_predict_and_save(model, batches, dev, pcsv,
                                                              num_mc_samples=Ni), 1)
                infer_sweep[name] = {
                    "value": round(Ni * Bi * nb / d, 2), "unit": "MC-samples/s",
                    "batch": Bi, "num_mc": Ni, "batches": nb, "sonar_px": S,
                    "optical_px": args.optical, "ms_per_batch": round(d / nb * 1e3, 2),
                    "sharding": "mc" if world > 1 else "none", "mc_chunk": ck,
                    "peak_hbm_gib": round(torch.cuda.max_memory_allocated(dev) / 2**30, 1)}
            except Exception as e:   # a leg that fails is reported; the headline still prints
                infer_sweep[name] = {"error": type(e).__name__, "detail": str(e)[:200]}
            finally:
                batches = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress("cpu baseline")
        cpu = cpu_baseline(args)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(triplets_s, 3), "unit": "triplets/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (random-init weights, MOPED rho; inputs resident in HBM)",
            "config": {"workload": ("configs[1]" if args.dtype == "fp32" else "configs[2] slice")
                                   + ": tri-modal BNN training step, 7 classes, "
                                   f"B={args.batch}/GPU {args.dtype}, num_mc={args.num_mc}, optical "
                                   f"{args.optical}px + bathy/SSS {args.sonar}px",
                       "global_batch": args.batch * world, "num_mc": args.num_mc,
                       "parallelism": f"dp{world}",
                       "grad_exchange": args.grad_exchange if world > 1 else None},
            "f32_math": f32_math if args.dtype == "fp32" else None,
            "fp32_exact_mfma": exact,
            "inference": infer, "infer_sweep": infer_sweep, "bf16_train": bf16,
            "train_sweep": sweep, "configs0_unimodal": uni, "roofline": roof, "comm": comm,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
