mkdir -p gpurun_out/r6
export TMPDIR=/tmp
O=gpurun_out/r6
for z in 0 1 2; do
MAUV_CENTRE_MIN_Z=$z timeout -k 10 300 python -u -m pytest -x -q -rP --timeout 250 --timeout-method thread "tests/test_dropin_gpu.py::test_g6_predict_under_autocast" > $O/g6_z$z.log 2>&1; echo "z=$z rc=$?"; grep -E "max dev" $O/g6_z$z.log
done
MAUV_CENTRE_Y=0 timeout -k 10 300 python -u -m pytest -x -q -rP --timeout 250 --timeout-method thread "tests/test_dropin_gpu.py::test_g6_predict_under_autocast" > $O/g6_off.log 2>&1; echo "off rc=$?"; grep -E "max dev" $O/g6_off.log
MAUV_CENTRE_MIN_Z=1 timeout -k 10 600 python -u tools/pred_bisect.py --seeds 8 > $O/pred_sweep_centred_z1.log 2>&1; r=$?; tail -1 $O/pred_sweep_centred_z1.log; exit $r
