#!/bin/bash
# round-5 GPU call 15: conv_haloc16 (3x3 / stride-1 forwards over 128-512 channels through a
# chunked LDS row image) — its tests and the forward kernels' identity / chunking / parity tests,
# per-shape A/B against the implicit GEMM, then inference and bf16 training A/Bs
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c15; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 300 --timeout-method thread tests/test_haloc16_gpu.py tests/test_halo16_gpu.py tests/test_expand16_gpu.py tests/test_configs4_gpu.py tests/test_parity16_gpu.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; [ $r -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/haloc_ab.py --dtype bf16 > $O/ab_bf16.log 2>&1; r=$?; echo "ab bf16 rc=$r"; [ $r -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/haloc_ab.py --dtype f16 --B 256 > $O/ab_f16.log 2>&1; r=$?; echo "ab f16 rc=$r"; [ $r -eq 0 ] || exit 1
timeout -k 10 600 python -u tools/fold_ab.py --flag haloc16 --rounds 4 > $O/infer.log 2>&1; r=$?; echo "infer rc=$r"; [ $r -eq 0 ] || exit 1
timeout -k 10 600 python -u tools/fold_ab.py --train --dtype bf16 --flag haloc16 --rounds 3 > $O/train.log 2>&1; echo "train rc=$?"
