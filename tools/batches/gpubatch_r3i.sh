# round 3: backward fusions — BN-backward partials from the data-gradient epilogue (16-bit:
# operands prefetched two chunks ahead; fp32: the split kernel's direct-store epilogue), the
# residual gradient from mask bits (no dres tensor), the segmented BN-backward finalize:
# kernel + engine tests, then interleaved same-box A/Bs of the bf16 and fp32 steps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_bwd_fusion_gpu.py tests/test_kernels_gpu.py::test_bn_bwd_segmented_final tests/test_kernels_gpu.py::test_bn_fwd_bwd tests/test_kernels_gpu.py::test_bn_relu_mask_path_matches_output_path tests/test_kernels16_gpu.py::test_conv16_dgrad_bn_partials_epilogue -v -s --timeout 300 --timeout-method thread > gpurun_out/r3i_test.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert|cosine" gpurun_out/r3i_test.log | tail -30
[ $rc -eq 0 ] || { echo "tests rc=$rc: stop"; exit $rc; }
C="--no-infer --no-cpu-baseline --no-roofline --no-sweep --no-infer-sweep --no-bf16 --exact-steps 0 --steps 10 --warmup 3"
for r in 1 2; do
  for v in "0 0" "1 0" "0 1" "1 1"; do
    set -- $v
    MAUV_DGRAD_BN_EPI=$1 MAUV_RES_MASK=$2 timeout -k 10 300 python -u bench.py --dtype bf16 $C > gpurun_out/r3i_ab_$1$2_$r.log 2> gpurun_out/r3i_ab_$1$2_$r.err || { tail -5 gpurun_out/r3i_ab_$1$2_$r.err; exit 1; }
    echo "bf16 epi=$1 resmask=$2 round $r: $(grep -o '"value": [0-9.]*' gpurun_out/r3i_ab_$1$2_$r.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3i_ab_$1$2_$r.log | head -1)"
  done
done
for r in 1 2; do
  for v in "0 0" "1 1" "0 1"; do
    set -- $v
    MAUV_DGRAD_BN_EPI_F32=$1 MAUV_RES_MASK=$2 timeout -k 10 300 python -u bench.py $C > gpurun_out/r3i_f32_$1$2_$r.log 2> gpurun_out/r3i_f32_$1$2_$r.err || { tail -5 gpurun_out/r3i_f32_$1$2_$r.err; exit 1; }
    echo "fp32 epi=$1 resmask=$2 round $r: $(grep -o '"value": [0-9.]*' gpurun_out/r3i_f32_$1$2_$r.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3i_f32_$1$2_$r.log | head -1)"
  done
done
for v in 0 1; do
  MAUV_DGRAD_BN_EPI=$v MAUV_RES_MASK=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3i_prof_$v -o run -- python3 bench.py --dtype bf16 --no-infer --no-cpu-baseline --no-roofline --no-sweep --no-infer-sweep --no-bf16 --exact-steps 0 --steps 3 --warmup 1 > gpurun_out/r3i_prof_$v.log 2>&1 || { tail -5 gpurun_out/r3i_prof_$v.log; exit 1; }
  MAUV_DGRAD_BN_EPI_F32=$v MAUV_RES_MASK=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3i_proff_$v -o run -- python3 bench.py --no-infer --no-cpu-baseline --no-roofline --no-sweep --no-infer-sweep --no-bf16 --exact-steps 0 --steps 3 --warmup 1 > gpurun_out/r3i_proff_$v.log 2>&1 || { tail -5 gpurun_out/r3i_proff_$v.log; exit 1; }
done
echo done
