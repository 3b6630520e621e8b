# round 1c evidence: every GPU test, smoke(), kernel traces (fp32 step, bf16 step, f16
# inference), conv HBM traffic (PMC), default bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c_tests.log 2>&1 || { tail -30 gpurun_out/c_tests.log; exit 1; }
tail -n 2 gpurun_out/c_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c_smoke.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c_prof_fp32 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline > gpurun_out/c_prof_fp32.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c_prof_bf16 -o run -- python3 bench.py --dtype bf16 --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-bf16 --no-roofline > gpurun_out/c_prof_bf16.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c_prof_inf -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-bf16 --exact-steps 0 --no-roofline > gpurun_out/c_prof_inf.log 2>&1 || exit 1
B="bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/c_pmc_fetch -o run -- python3 $B > gpurun_out/c_pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/c_pmc_write -o run -- python3 $B > gpurun_out/c_pmc_write.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/c_bench.log 2>&1 || exit 1
tail -n 1 gpurun_out/c_bench.log
echo done
