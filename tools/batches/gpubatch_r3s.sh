# round 3, final state (2.17 + the BN finalize geometry): the full GPU suite and smoke(), PMC traffic of both conv families on this
# library (copied where bench.py reads it), the default bench line, serial kernel statistics of
# one fp32 and one bf16 step, and kernel statistics of the f16 inference leg
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3s_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r3s_tests.log | head; tail -5 gpurun_out/r3s_tests.log; exit 1; }
tail -1 gpurun_out/r3s_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s_smoke.log 2>&1 || { tail -20 gpurun_out/r3s_smoke.log; exit 1; }
tail -1 gpurun_out/r3s_smoke.log
B32="bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline --no-sweep"
B16="bench.py --dtype bf16 --steps 1 --warmup 0 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline --no-sweep"
MAUV_TRUNK_STREAMS=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3s_pmc_f32_fetch -o run -- python3 $B32 > gpurun_out/r3s_pmc_f32_fetch.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/r3s_pmc_f32_write -o run -- python3 $B32 > gpurun_out/r3s_pmc_f32_write.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3s_pmc_b16_fetch -o run -- python3 $B16 > gpurun_out/r3s_pmc_b16_fetch.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/r3s_pmc_b16_write -o run -- python3 $B16 > gpurun_out/r3s_pmc_b16_write.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/r3s_pmc_f32_fetch gpurun_out/r3s_pmc_f32_write gpurun_out/round3s_conv_traffic.json > gpurun_out/r3s_pmc_f32_summary.txt || exit 1
python3 tools/pmc_traffic.py gpurun_out/r3s_pmc_b16_fetch gpurun_out/r3s_pmc_b16_write gpurun_out/round3s_bf16_conv_traffic.json > gpurun_out/r3s_pmc_b16_summary.txt || exit 1
cp gpurun_out/round3s_conv_traffic.json gpurun_out/round3s_bf16_conv_traffic.json profiles/ || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/round3s_bench.log 2>&1 || { tail -20 gpurun_out/round3s_bench.log; exit 1; }
tail -1 gpurun_out/round3s_bench.log > gpurun_out/round3s_bench.json
python3 -c "import json;d=json.load(open('gpurun_out/round3s_bench.json'));print(d['value'], d['bf16_train']['value'], d['inference']['value'], d['roofline']['frac'], d['roofline']['traffic_matches_library'], d['bf16_train']['roofline']['frac'], d['bf16_train']['roofline']['traffic_matches_library'])"
C="--no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer --no-bf16"
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s_st32 -o run -- python3 bench.py --steps 2 --warmup 1 $C > gpurun_out/r3s_st32.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s_st16 -o run -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 $C > gpurun_out/r3s_st16.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s_inf -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer-sweep --no-bf16 --no-infer-fp32 > gpurun_out/r3s_inf.log 2>&1 || exit 1
echo done
