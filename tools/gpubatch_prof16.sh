# kernel traces: bf16 training step, f16 autocast MC inference
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bf16 -o run -- python3 bench.py --dtype bf16 --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-bf16 --no-roofline > gpurun_out/prof_bf16.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_inf -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-bf16 --exact-steps 0 --no-roofline > gpurun_out/prof_inf.log 2>&1 || exit 1
echo done
