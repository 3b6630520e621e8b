#!/bin/bash
# round-5 GPU call 6: fp32 BN-backward partials from the staged data-gradient epilogue — kernel /
# fusion / model tests, same-box A/B of the fp32 step, bench line
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5c6; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 "$@" > $O/$n.log 2>&1; local r=$?; echo "$n rc=$r"; [ $r -le 1 ]; }
run tests 700 python -u -m pytest -v -rP --timeout 300 --timeout-method thread tests/test_kernels16_gpu.py tests/test_bwd_fusion_gpu.py tests/test_model_gpu.py tests/test_kernels_gpu.py tests/test_shipped_gpu.py::test_configs1_fp32_step_b64 &&
run ab 600 python -u tools/fold_ab.py --train --dtype fp32 --flag BWD_PARTIALS_F32 --rounds 4 --steps 10 &&
run bench 900 python -u bench.py
