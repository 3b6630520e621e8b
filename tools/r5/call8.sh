#!/bin/bash
# round-5 GPU call 8: the weight-stationary 16-bit expansion forwards (conv_expand16.hip) —
# kernel tests against conv_pipe16, per-shape A/B, bf16 step and f16 inference A/Bs
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c8; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 "$@" > $O/$n.log 2>&1; local r=$?; echo "$n rc=$r"; [ $r -eq 0 ]; }
run tests 300 python -u -m pytest -x -v -rP --timeout 120 --timeout-method thread tests/test_expand16_gpu.py || exit 1
run shapes_bf16 300 python -u tools/expand_ab.py --dtype bf16 --G 5 --B 64 --rounds 3 || exit 1
run shapes_f16 400 python -u tools/expand_ab.py --dtype f16 --G 20 --B 256 --rounds 2 || exit 1
run train 500 python -u tools/fold_ab.py --train --dtype bf16 --flag expand16 --rounds 4 --steps 10 || exit 1
run infer 500 python -u tools/fold_ab.py --flag expand16 --rounds 3 || exit 1
echo done
