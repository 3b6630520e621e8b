# full training step kernel trace (split fp32 default) for profiles/
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_step -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline > gpurun_out/prof_step.log 2>&1 || exit 1
echo done
