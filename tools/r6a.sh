mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/pred_bisect.py > gpurun_out/r6/pred_bisect.log 2>&1; r=$?; tail -22 gpurun_out/r6/pred_bisect.log; [ $r -eq 0 ] || exit 1
timeout -k 10 600 python -u tools/pred_bisect.py --seeds 8 > gpurun_out/r6/pred_sweep.log 2>&1; r=$?; tail -10 gpurun_out/r6/pred_sweep.log; [ $r -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 500 --timeout-method thread tests/test_model_gpu.py::test_predict_fp32_fitted_full_size tests/test_shipped_gpu.py::test_configs1_fp32_step_b64 > gpurun_out/r6/new_tests.log 2>&1; r=$?; grep -E "vs float64|max \|d\||whole-gradient|passed|failed|Error|assert" gpurun_out/r6/new_tests.log | tail -40; exit $r
