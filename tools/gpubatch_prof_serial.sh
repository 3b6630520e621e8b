# kernel traces with the trunks serialised (MAUV_TRUNK_STREAMS=0): per-kernel durations as the
# bench's roofline step measures them
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export MAUV_TRUNK_STREAMS=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c_prof_fp32s -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline > gpurun_out/c_prof_fp32s.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c_prof_bf16s -o run -- python3 bench.py --dtype bf16 --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-bf16 --no-roofline > gpurun_out/c_prof_bf16s.log 2>&1 || exit 1
echo done
