# round 3: weight-gradient split count priced with its fp32 slab bytes (MAUV_WGRAD_SPLITS=2, new
# default) against the round-filling rule (=1): wgrad-touching GPU tests under the new rule,
# per-shape wgrad totals, interleaved bf16 / fp32 training legs; one bf16 step's kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "wgrad or weight or grad or train or reparam" > gpurun_out/r3m_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r3m_tests.log | head; tail -5 gpurun_out/r3m_tests.log; exit 1; }
tail -1 gpurun_out/r3m_tests.log
for m in 1 2; do
  MAUV_WGRAD_SPLITS=$m timeout -k 10 300 python -u tools/conv_bench.py --dtype bf16 --fused --only wgrad --top 0 --reps 10 > gpurun_out/r3m_cb_$m.txt 2>&1 || { tail -5 gpurun_out/r3m_cb_$m.txt; exit 1; }
  echo "mode $m bf16: $(grep 'TOTAL wgrad' gpurun_out/r3m_cb_$m.txt)"
done
B16="--no-cpu-baseline --no-roofline --no-sweep --no-infer --no-bf16 --exact-steps 0 --steps 8 --warmup 2 --dtype bf16"
B32="--no-cpu-baseline --no-roofline --no-sweep --no-infer --no-bf16 --exact-steps 0 --steps 6 --warmup 2"
for r in 1 2; do
  for m in 1 2; do
    MAUV_WGRAD_SPLITS=$m timeout -k 10 300 python -u bench.py $B16 > gpurun_out/r3m_b16_${m}_$r.log 2>&1 || { tail -5 gpurun_out/r3m_b16_${m}_$r.log; exit 1; }
    MAUV_WGRAD_SPLITS=$m timeout -k 10 300 python -u bench.py $B32 > gpurun_out/r3m_b32_${m}_$r.log 2>&1 || { tail -5 gpurun_out/r3m_b32_${m}_$r.log; exit 1; }
    echo "mode $m round $r: bf16 $(tail -1 gpurun_out/r3m_b16_${m}_$r.log | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["value"])') fp32 $(tail -1 gpurun_out/r3m_b32_${m}_$r.log | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["value"])')"
  done
done
for m in 1 2; do
  MAUV_WGRAD_SPLITS=$m MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3m_st16_$m -o run -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer --no-bf16 > gpurun_out/r3m_st16_$m.log 2>&1 || exit 1
done
echo done
