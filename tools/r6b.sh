# round-6 call b: f16 rounding points, the new parity tests + the route-refactor tests, the 1x1
# table against rocBLAS, then (last: it may fault) torch.bmm alone at the round-5 fault shape
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
O=gpurun_out/r6
timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 500 --timeout-method thread tests/test_model_gpu.py::test_predict_fp32_fitted_full_size tests/test_shipped_gpu.py::test_configs1_fp32_step_b64 > $O/b_tests.log 2>&1; r=$?; grep -E "vs float64|max \|d\||whole-gradient|passed|failed|Error" $O/b_tests.log | tail -30; [ $r -eq 0 ] || exit 1
timeout -k 10 400 python -u tools/f16_rounding_points.py > $O/f16_rounding_points.log 2>&1; r=$?; tail -14 $O/f16_rounding_points.log; [ $r -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/fwd_ab.py --only1x1 --min-k 64 --blas rocblas --rounds 2 > $O/fwd_1x1_bf16_G5_B64_rocblas.txt 2>&1; r=$?; tail -3 $O/fwd_1x1_bf16_G5_B64_rocblas.txt; [ $r -eq 0 ] || exit 1
timeout -k 10 120 python -u tools/bmm_fault_probe.py cublaslt > $O/bmm_fault_probe.log 2>&1; r=$?; cat $O/bmm_fault_probe.log | tail -5; exit $r
