# round 1c: inference kernel trace + the default bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c_prof_inf -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-bf16 --exact-steps 0 --no-roofline > gpurun_out/c_prof_inf.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/c_bench.log 2>&1 || exit 1
tail -n 1 gpurun_out/c_bench.log | cut -c1-700
echo done
