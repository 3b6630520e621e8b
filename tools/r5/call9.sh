#!/bin/bash
# round-5 GPU call 9: conv_expand16 routed where it measured faster (K = 128; K = 256 with >= 8
# row pairs per block) — tests, bf16 step and f16 inference A/Bs of the default routing
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c9; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 "$@" > $O/$n.log 2>&1; local r=$?; echo "$n rc=$r"; [ $r -eq 0 ]; }
run tests 300 python -u -m pytest -x -v -rP --timeout 120 --timeout-method thread tests/test_expand16_gpu.py tests/test_kernels16_gpu.py || exit 1
run train 500 python -u tools/fold_ab.py --train --dtype bf16 --flag expand16 --rounds 4 --steps 10 || exit 1
run infer 600 python -u tools/fold_ab.py --flag expand16 --rounds 4 || exit 1
echo done
