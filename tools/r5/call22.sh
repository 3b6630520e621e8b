#!/bin/bash
# round-5 GPU call 22: conv_haloc16 data gradients (3x3 / stride-1, 128-512 channels) — its
# tests and the data-gradient / fusion / chunking / parity tests, then the bf16 step A/B of
# mode 1 (forwards + data gradients) against mode 3 (forwards only), and the per-shape timing
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c22; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_haloc16_gpu.py tests/test_kernels16_gpu.py tests/test_bwd_fusion_gpu.py tests/test_configs4_gpu.py tests/test_model16_gpu.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; [ $r -eq 0 ] || exit 1
timeout -k 10 600 python -u tools/fold_ab.py --train --dtype bf16 --flag haloc16:3 --rounds 3 > $O/train.log 2>&1; r=$?; echo "train rc=$r"; [ $r -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/step_shapes.py --dtype bf16 --top 40 > $O/shapes_bf16.txt 2>&1; echo "shapes rc=$?"
