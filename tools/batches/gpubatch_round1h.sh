# round-1h evidence (BN partial pass at 32 rows per thread): 64-row A/B, every GPU test, smoke, kernel traces, default bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fin_tests.log 2>&1 || { tail -30 gpurun_out/fin_tests.log; exit 1; }
tail -n 1 gpurun_out/fin_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 || exit 1
tail -n 2 gpurun_out/fin_smoke.log
for v in 32 64; do
MAUV_BN_PARTIAL_RPT=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline --no-infer > gpurun_out/r3_b.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/r3_b.log').read().strip().splitlines()[-1]);print('partial=$v', d['value'], d['bf16_train']['value'])"
done
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin_prof_fp32s -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline > gpurun_out/fin_prof_fp32s.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin_prof_bf16s -o run -- python3 bench.py --dtype bf16 --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-bf16 --no-roofline > gpurun_out/fin_prof_bf16s.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/fin_bench.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/fin_bench.log').read().strip().splitlines()[-1]);print(d['value'], d['inference']['value'], d['bf16_train']['value'], d['fp32_exact_mfma']['value'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['cpu_baseline']['value'])"
echo done
