mkdir -p gpurun_out/r6
export TMPDIR=/tmp
O=gpurun_out/r6
timeout -k 10 500 python -u tools/f16_rounding_points.py > $O/f16_rounding_points2.log 2>&1; r=$?; tail -15 $O/f16_rounding_points2.log; exit $r
