#!/bin/bash
# round-5 GPU call 14: canonical 16-bit forward statistics (64-row halves merged by Chan's
# formula, shared by every 16-bit forward kernel) — kernel identity tests, configs[4] chunking,
# 16-bit parity, then the expand16 K = 256 routing's inference A/B
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c14; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v -rP --timeout 300 --timeout-method thread tests/test_expand16_gpu.py tests/test_big16_gpu.py tests/test_halo16_gpu.py tests/test_fold_gpu.py tests/test_kernels16_gpu.py tests/test_configs4_gpu.py tests/test_parity16_gpu.py tests/test_dropin_gpu.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; [ $r -eq 0 ] || exit 1
timeout -k 10 600 python -u tools/fold_ab.py --flag expand16 --rounds 4 > $O/infer.log 2>&1; echo "infer rc=$?"
