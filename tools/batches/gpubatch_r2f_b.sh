# round-2 evidence, part F2: the r2f batch after its test/smoke half (run separately by gpubatch_r2final_a.sh)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_f32_math_gpu.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r2f_f32_tests.log 2>&1 || { tail -20 gpurun_out/r2f_f32_tests.log; exit 1; }
tail -1 gpurun_out/r2f_f32_tests.log
B32="bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline"
B16="bench.py --dtype bf16 --steps 1 --warmup 0 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline"
MAUV_TRUNK_STREAMS=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/f_pmc32f -o run -- python3 $B32 > gpurun_out/f_pmc32f.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/f_pmc32w -o run -- python3 $B32 > gpurun_out/f_pmc32w.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/f_pmc16f -o run -- python3 $B16 > gpurun_out/f_pmc16f.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/f_pmc16w -o run -- python3 $B16 > gpurun_out/f_pmc16w.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/f_pmc32f gpurun_out/f_pmc32w gpurun_out/round2f_conv_traffic.json conv_f32 > gpurun_out/f_pmc32.txt || exit 1
python3 tools/pmc_traffic.py gpurun_out/f_pmc16f gpurun_out/f_pmc16w gpurun_out/round2f_bf16_conv_traffic.json conv_h16 > gpurun_out/f_pmc16.txt || exit 1
cp gpurun_out/round2f_conv_traffic.json gpurun_out/round2f_bf16_conv_traffic.json profiles/
head -3 gpurun_out/f_pmc32.txt gpurun_out/f_pmc16.txt
timeout -k 10 600 python -u bench.py > gpurun_out/round2f_bench.log 2>&1 || { tail -20 gpurun_out/round2f_bench.log; exit 1; }
tail -1 gpurun_out/round2f_bench.log > gpurun_out/round2f_bench.json
C="--no-cpu-baseline --exact-steps 0 --no-roofline"
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f_st32 -o run -- python3 bench.py --steps 2 --warmup 1 $C --no-infer --no-bf16 > gpurun_out/f_st32.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f_st16 -o run -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 $C --no-infer --no-bf16 > gpurun_out/f_st16.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f_stinf -o run -- python3 bench.py --steps 1 --warmup 0 $C --no-bf16 --no-infer-fp32 > gpurun_out/f_stinf.log 2>&1 || exit 1
echo done
