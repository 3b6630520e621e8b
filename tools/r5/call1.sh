#!/bin/bash
# round-5 GPU call 1: new DMA-128 forward parity, shipped-size parity, autocast resolution sweep,
# per-shape forward A/B, host fill/copy sites.  Stops at the first crash / timeout (rc > 1).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5c1; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 "$@" > $O/$n.log 2>&1; local r=$?; echo "$n rc=$r"; [ $r -le 1 ]; }
run tests 600 python -u -m pytest -v -rP --timeout 300 --timeout-method thread tests/test_big16_gpu.py tests/test_shipped_gpu.py &&
run explore 600 python -u tools/parity16_explore.py 64,64,8,2 64,64,16,2 64,64,32,2 96,96,16,2 128,128,16,2 224,256,8,2 &&
run fwd_bf16 300 python -u tools/fwd_ab.py --dtype bf16 --G 5 --B 64 --min-k 256 --rounds 3 &&
run fwd_f16 400 python -u tools/fwd_ab.py --dtype f16 --G 20 --B 256 --min-k 256 --rounds 2 &&
run hostops 300 python -u tools/host_ops.py --dtype bf16
