#!/bin/bash
# round-5 GPU call 19: conv_haloc16 with the nine taps unrolled (the default form) — its tests,
# configs[4] chunking, then f16 inference and bf16 step A/Bs against the implicit GEMM
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c19; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 300 --timeout-method thread tests/test_haloc16_gpu.py tests/test_configs4_gpu.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; [ $r -eq 0 ] || exit 1
timeout -k 10 600 python -u tools/fold_ab.py --flag haloc16 --rounds 4 > $O/infer.log 2>&1; r=$?; echo "infer rc=$r"; [ $r -eq 0 ] || exit 1
timeout -k 10 600 python -u tools/fold_ab.py --train --dtype bf16 --flag haloc16 --rounds 3 > $O/train.log 2>&1; echo "train rc=$?"
