#!/bin/bash
# round-5 GPU call 3: fp32 dgrad staged epilogue — kernel tests, shipped tests, A/B on the fp32
# leg, in-step shapes; f16 / fitted bf16 autocast resolution
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5c3; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 "$@" > $O/$n.log 2>&1; local r=$?; echo "$n rc=$r"; [ $r -le 1 ]; }
run ktests 600 python -u -m pytest -v -rP --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_bwd_fusion_gpu.py tests/test_shipped_gpu.py::test_configs1_fp32_step_b64 &&
run ab 1000 bash tools/r5/ab_lib.sh $O/ab 2 multimodal-auv_amd/mauv/libmauv_hip_base.so -- --steps 10 --warmup 2 --no-infer --no-bf16 --no-sweep --exact-steps 0 --no-cpu-baseline --no-roofline &&
run steps32 300 python -u tools/step_shapes.py --dtype fp32 --top 30 &&
run explore16 400 python -u tools/parity16_explore.py --dtype f16 64,64,8,2 64,64,32,2 224,256,8,2 &&
run explorefit 400 python -u tools/parity16_explore.py --dtype bf16 --fit 20 64,64,8,2 64,64,32,2
