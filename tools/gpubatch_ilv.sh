set -o pipefail
mkdir -p gpurun_out
for v in "0 0" "4 0" "6 0" "0 1"; do
  set -- $v
  MAUV_SPLIT_ILV=$1 MAUV_SPLIT_DEEP=$2 timeout -k 10 300 python -u tools/conv_bench.py --reps 3 --top 3 --fused > gpurun_out/ilv_$1_$2.log 2>&1 || exit 1
done
MAUV_SPLIT_DEEP=1 timeout -k 10 300 python -u -m pytest -x -q tests/test_f32_math_gpu.py > gpurun_out/ilv_deep_test.log 2>&1 || exit 1
echo done
