# whole-grid XCD-aware tile order (MAUV_XCD_GRID, conv_common.h conv_block_tile) and the
# round-filling weight-gradient split count (MAUV_WGRAD_SPLITS, conv_gemm.hip) against the
# round-1 rules: conv kernel parity, per-family conv totals, training + inference A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernels16_gpu.py tests/test_f32_math_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s3x_tests.log 2>&1 || { tail -30 gpurun_out/s3x_tests.log; exit 1; }
tail -1 gpurun_out/s3x_tests.log
for v in "0 0" "1 0" "1 1"; do
  set -- $v
  for dt in fp32 bf16; do
    MAUV_XCD_GRID=$1 MAUV_WGRAD_SPLITS=$2 timeout -k 10 200 python -u tools/conv_bench.py --dtype $dt --fused --top 0 > gpurun_out/s3x_cb_${dt}_$1$2.txt 2>&1 || exit 1
    echo "grid=$1 splits=$2 $dt"; grep TOTAL gpurun_out/s3x_cb_${dt}_$1$2.txt
  done
done
B="--no-cpu-baseline --exact-steps 0 --no-roofline"
for v in "0 0" "1 1" "0 0" "1 1"; do
  set -- $v
  MAUV_XCD_GRID=$1 MAUV_WGRAD_SPLITS=$2 timeout -k 10 300 python -u bench.py $B --no-infer > gpurun_out/s3x_tr.log 2>&1 || { tail -5 gpurun_out/s3x_tr.log; exit 1; }
  echo "grid=$1 splits=$2 train"; tail -1 gpurun_out/s3x_tr.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['bf16_train']['value'])"
done
for v in 0 1; do
  MAUV_XCD_GRID=$v timeout -k 10 300 python -u bench.py $B --no-bf16 --no-infer-fp32 --steps 1 --warmup 1 > gpurun_out/s3x_inf_$v.log 2>&1 || { tail -5 gpurun_out/s3x_inf_$v.log; exit 1; }
  echo "grid=$v infer"; tail -1 gpurun_out/s3x_inf_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['inference']['value'])"
done
