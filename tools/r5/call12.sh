#!/bin/bash
# round-5 GPU call 12: the parity16 tests after the expand16 routing fix (per-tensor bars moved
# to the resolved shapes) and the configs[4] chunk-exactness test
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c12; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v -rP --timeout 300 --timeout-method thread tests/test_parity16_gpu.py tests/test_configs4_gpu.py tests/test_expand16_gpu.py > $O/tests.log 2>&1; echo "tests rc=$?"
