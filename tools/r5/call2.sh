#!/bin/bash
# round-5 GPU call 2: retry of call 1's failing tests, gate tests, autocast resolution sweep,
# in-step per-shape conv tables (fp32, bf16).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5c2; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 "$@" > $O/$n.log 2>&1; local r=$?; echo "$n rc=$r"; [ $r -le 1 ]; }
run tests 900 python -u -m pytest -v -rP --timeout 400 --timeout-method thread tests/test_big16_gpu.py tests/test_shipped_gpu.py tests/test_step_gate_gpu.py &&
run explore 600 python -u tools/parity16_explore.py 64,64,8,2 64,64,16,2 64,64,32,2 96,96,16,2 128,128,16,2 224,256,8,2 &&
run steps32 300 python -u tools/step_shapes.py --dtype fp32 --top 60 &&
run steps16 300 python -u tools/step_shapes.py --dtype bf16 --top 60
