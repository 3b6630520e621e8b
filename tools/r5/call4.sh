#!/bin/bash
# round-5 GPU call 4: per-shape fp32 tables of the split variants, in-step shapes, autocast
# resolution of f16 / a fitted bf16 model
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5c4; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 "$@" > $O/$n.log 2>&1; local r=$?; echo "$n rc=$r"; [ $r -le 1 ]; }
run cb0 200 env MAUV_SPLIT_OPTS=0 python -u tools/conv_bench.py --dtype fp32 --top 300 --fused &&
run cb1 200 env MAUV_SPLIT_OPTS=1 python -u tools/conv_bench.py --dtype fp32 --top 300 --fused &&
run cb2 200 env MAUV_SPLIT_OPTS=2 python -u tools/conv_bench.py --dtype fp32 --top 300 --fused &&
run steps32 300 python -u tools/step_shapes.py --dtype fp32 --top 30 &&
run explore16 400 python -u tools/parity16_explore.py --dtype f16 64,64,8,2 64,64,32,2 224,256,8,2 &&
run explorefit 400 python -u tools/parity16_explore.py --dtype bf16 --fit 20 64,64,8,2 64,64,32,2
