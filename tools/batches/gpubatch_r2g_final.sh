# round 2g, final state: the full GPU suite, smoke(), the default bench line and serial kernel
# statistics of one fp32 and one bf16 step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r2gf_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r2gf_tests.log | head; tail -5 gpurun_out/r2gf_tests.log; exit 1; }
tail -1 gpurun_out/r2gf_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2gf_smoke.log 2>&1 || { tail -20 gpurun_out/r2gf_smoke.log; exit 1; }
tail -1 gpurun_out/r2gf_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/round2g_final_bench.log 2>&1 || { tail -20 gpurun_out/round2g_final_bench.log; exit 1; }
tail -1 gpurun_out/round2g_final_bench.log > gpurun_out/round2g_final_bench.json
python3 -c "import json;d=json.load(open('gpurun_out/round2g_final_bench.json'));print(d['value'], d['bf16_train']['value'], d['inference']['value'], d['roofline']['frac'], d['bf16_train']['roofline']['frac'], json.dumps(d['train_sweep']))"
C="--no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep"
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gf_st32 -o run -- python3 bench.py --steps 2 --warmup 1 $C --no-infer --no-bf16 > gpurun_out/gf_st32.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gf_st16 -o run -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 $C --no-infer --no-bf16 > gpurun_out/gf_st16.log 2>&1 || exit 1
echo done
