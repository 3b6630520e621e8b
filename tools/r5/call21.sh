#!/bin/bash
# round-5 GPU call 21: fp32 data-gradient epilogue parking the accumulators first with four
# chunks in flight (and one staging pass for the short-K BN-partials kernel) — fp32 kernel /
# fusion tests, in-step shapes of both libraries, then fp32 bench legs interleaved (base = the
# previous library)
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c21; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_bwd_fusion_gpu.py tests/test_model_gpu.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; [ $r -eq 0 ] || exit 1
MAUV_LIB=multimodal-auv_amd/mauv/libmauv_hip_base.so timeout -k 10 300 python -u tools/step_shapes.py --top 30 > $O/shapes_base.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/step_shapes.py --top 30 > $O/shapes_new.txt 2>&1 || exit 1
grep TOTAL $O/shapes_base.txt $O/shapes_new.txt
bash tools/r5/ab_lib.sh $O/ab 4 multimodal-auv_amd/mauv/libmauv_hip_base.so -- --steps 10 --warmup 3 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline --no-sweep
