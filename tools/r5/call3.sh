#!/bin/bash
# round-5 GPU call 3: fp32 epilogues / split variants — kernel + model tests, interleaved A/B of
# the fp32 training leg (base library vs the variants)
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5c3; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 "$@" > $O/$n.log 2>&1; local r=$?; echo "$n rc=$r"; [ $r -le 1 ]; }
run ktests 600 python -u -m pytest -v -rP --timeout 300 --timeout-method thread tests/test_dropin_gpu.py::test_g6_predict_under_autocast &&
run ab 700 bash tools/r5/ab_arms.sh $O/ab 2 "base|MAUV_LIB=multimodal-auv_amd/mauv/libmauv_hip_base.so" "dgrad|MAUV_SPLIT_OPTS=4" "both|MAUV_SPLIT_OPTS=0" "w4|MAUV_SPLIT_OPTS=2" "fl|MAUV_SPLIT_OPTS=1" -- --steps 10 --warmup 2 --no-infer --no-bf16 --no-sweep --exact-steps 0 --no-cpu-baseline --no-roofline
