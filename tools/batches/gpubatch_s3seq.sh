# RECORD ONLY: the switch MAUV_SPLIT_SHORT_K_DGRAD and the variant it selected were measured (DESIGN.md cites the result)
# and removed from the code; this script no longer reproduces that A/B.
# short-K (SEQ) split-fp32 kernels for the data gradient (MAUV_SPLIT_SHORT_K_DGRAD) and a
# forward threshold of 512 (MAUV_SPLIT_SHORT_K): conv totals and fp32 training A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 env MAUV_SPLIT_SHORT_K_DGRAD=512 python -u -m pytest tests/test_kernels_gpu.py tests/test_f32_math_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s3q_tests.log 2>&1 || { tail -30 gpurun_out/s3q_tests.log; exit 1; }
tail -1 gpurun_out/s3q_tests.log
for v in "256 0" "256 256" "256 512" "512 0"; do
  set -- $v
  MAUV_SPLIT_SHORT_K=$1 MAUV_SPLIT_SHORT_K_DGRAD=$2 timeout -k 10 200 python -u tools/conv_bench.py --dtype fp32 --fused --only fwd,dgrad --top 0 > gpurun_out/s3q_cb_$1_$2.txt 2>&1 || exit 1
  echo "sk=$1 skd=$2"; grep TOTAL gpurun_out/s3q_cb_$1_$2.txt
done
B="--no-cpu-baseline --exact-steps 0 --no-roofline --no-infer --no-bf16"
for v in 0 256 512 0 256 512; do
  MAUV_SPLIT_SHORT_K_DGRAD=$v timeout -k 10 300 python -u bench.py $B > gpurun_out/s3q_tr.log 2>&1 || { tail -5 gpurun_out/s3q_tr.log; exit 1; }
  echo "skd=$v train $(tail -1 gpurun_out/s3q_tr.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
