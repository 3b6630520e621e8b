# round 3 evidence on the current library: PMC traffic of both conv families (separate
# FETCH_SIZE / WRITE_SIZE passes, trunks serial) copied where bench.py reads it, then the default
# bench line (its roofline.traffic now from this same library), then serial kernel statistics of
# one fp32 and one bf16 step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B32="bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline --no-sweep"
B16="bench.py --dtype bf16 --steps 1 --warmup 0 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline --no-sweep"
MAUV_TRUNK_STREAMS=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3_pmc_f32_fetch -o run -- python3 $B32 > gpurun_out/r3_pmc_f32_fetch.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/r3_pmc_f32_write -o run -- python3 $B32 > gpurun_out/r3_pmc_f32_write.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3_pmc_b16_fetch -o run -- python3 $B16 > gpurun_out/r3_pmc_b16_fetch.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/r3_pmc_b16_write -o run -- python3 $B16 > gpurun_out/r3_pmc_b16_write.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/r3_pmc_f32_fetch gpurun_out/r3_pmc_f32_write gpurun_out/round3_conv_traffic.json > gpurun_out/r3_pmc_f32_summary.txt || exit 1
python3 tools/pmc_traffic.py gpurun_out/r3_pmc_b16_fetch gpurun_out/r3_pmc_b16_write gpurun_out/round3_bf16_conv_traffic.json > gpurun_out/r3_pmc_b16_summary.txt || exit 1
cp gpurun_out/round3_conv_traffic.json gpurun_out/round3_bf16_conv_traffic.json profiles/ || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/round3_bench.log 2>&1 || { tail -20 gpurun_out/round3_bench.log; exit 1; }
tail -1 gpurun_out/round3_bench.log > gpurun_out/round3_bench.json
python3 -c "import json;d=json.load(open('gpurun_out/round3_bench.json'));print(d['value'], d['bf16_train']['value'], d['inference']['value'], d['roofline']['frac'], d['roofline']['traffic_matches_library'], d['bf16_train']['roofline']['frac'])"
C="--no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer --no-bf16"
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_st32 -o run -- python3 bench.py --steps 2 --warmup 1 $C > gpurun_out/r3_st32.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_st16 -o run -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 $C > gpurun_out/r3_st16.log 2>&1 || exit 1

timeout -k 10 300 python -u tools/conv_bench.py --dtype bf16 --fused --top 80 > gpurun_out/r3_convbench_bf16.txt 2>&1 || exit 1
tail -4 gpurun_out/r3_convbench_bf16.txt
echo done
