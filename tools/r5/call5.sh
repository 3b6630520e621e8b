#!/bin/bash
# round-5 GPU call 5: the resolved 16-bit gradient tests (twice: run-to-run spread of autocast),
# the f16 fitted sweep, kernel tests after the split-variant removal, bench default line
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5c5; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 "$@" > $O/$n.log 2>&1; local r=$?; echo "$n rc=$r"; [ $r -le 1 ]; }
run explorefit16 300 python -u tools/parity16_explore.py --dtype f16 --fit 20 64,64,8,2 64,64,32,2 &&
run p16a 600 python -u -m pytest -v -rP --timeout 300 --timeout-method thread tests/test_parity16_gpu.py &&
run p16b 400 python -u -m pytest -v -rP --timeout 300 --timeout-method thread tests/test_parity16_gpu.py -k resolved &&
run ktests 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_f32_math_gpu.py tests/test_bwd_fusion_gpu.py &&
run bench 900 python -u bench.py
