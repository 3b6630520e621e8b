#!/bin/bash
# round-5 GPU call 16: conv_haloc16 with 64 x 64 wave tiles (mode 1) beside the 32 x 64 form
# (mode 2) — tests, per-shape A/B of modes 0 / 1 / 2, inference A/B of mode 1 against 0
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c16; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 300 --timeout-method thread tests/test_haloc16_gpu.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; [ $r -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/haloc_ab.py --dtype bf16 > $O/ab_bf16.log 2>&1; r=$?; echo "ab bf16 rc=$r"; [ $r -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/haloc_ab.py --dtype f16 --B 256 > $O/ab_f16.log 2>&1; r=$?; echo "ab f16 rc=$r"; [ $r -eq 0 ] || exit 1
timeout -k 10 600 python -u tools/fold_ab.py --flag haloc16 --rounds 4 > $O/infer.log 2>&1; echo "infer rc=$?"
