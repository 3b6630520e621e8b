# round-6 call d: centred 16-bit storage — its kernel tests, the 16-bit parity / route tests,
# then the predictor sweep over 8 seeds and the seed-0 bisect on the centred library
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
O=gpurun_out/r6
timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 300 --timeout-method thread tests/test_centre16_gpu.py tests/test_fold_gpu.py tests/test_kernels16_gpu.py tests/test_abi_host.py tests/test_big16_gpu.py tests/test_expand16_gpu.py tests/test_haloc16_gpu.py tests/test_halo16_gpu.py > $O/d_tests.log 2>&1; r=$?; grep -E "centred|passed|failed|Error" $O/d_tests.log | tail -30; [ $r -eq 0 ] || exit 1
timeout -k 10 600 python -u tools/pred_bisect.py --seeds 8 > $O/pred_sweep_centred.log 2>&1; r=$?; tail -10 $O/pred_sweep_centred.log; [ $r -eq 0 ] || exit 1
timeout -k 10 400 python -u tools/f16_rounding_points.py > $O/f16_rounding_points_centred.log 2>&1; r=$?; tail -3 $O/f16_rounding_points_centred.log; exit $r
