# HBM traffic of the conv family (two PMC passes over one training step)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 $B > gpurun_out/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 $B > gpurun_out/pmc_write.log 2>&1 || exit 1
echo done
