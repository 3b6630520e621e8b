# per-kernel breakdown: bf16 step, fp32 step (trunks serial) and one f16 inference batch
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export MAUV_TRUNK_STREAMS=0
C="--no-cpu-baseline --exact-steps 0 --no-roofline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2p_b16 -o run -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 $C --no-infer --no-bf16 > gpurun_out/r2p_b16.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2p_f32 -o run -- python3 bench.py --steps 2 --warmup 1 $C --no-infer --no-bf16 > gpurun_out/r2p_f32.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2p_inf -o run -- python3 bench.py --steps 1 --warmup 0 $C --no-bf16 --no-infer-fp32 > gpurun_out/r2p_inf.log 2>&1 || exit 1
find gpurun_out/r2p_b16 gpurun_out/r2p_f32 gpurun_out/r2p_inf -name "*kernel_stats.csv"
