# round 3: short-K kernels for the data gradients (MAUV_DGRAD_SHORT=1) — kernel parity under
# the switch, per-shape data-gradient timings of both families with and without it, then an
# interleaved same-box A/B of the fp32 and bf16 training steps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MAUV_DGRAD_SHORT=1 timeout -k 10 400 python -u -m pytest tests/test_kernels16_gpu.py::test_conv16_fwd_dgrad_wgrad tests/test_kernels_gpu.py::test_conv_fwd_dgrad_wgrad tests/test_kernels_gpu.py::test_dgrad_accumulate_into_dx tests/test_bwd_fusion_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3ds_test.log 2>&1 || { tail -30 gpurun_out/r3ds_test.log; exit 1; }
tail -2 gpurun_out/r3ds_test.log
for v in 0 1; do
  for d in fp32 bf16; do
    MAUV_DGRAD_SHORT=$v timeout -k 10 300 python -u tools/conv_bench.py --dtype $d --only dgrad --top 400 > gpurun_out/r3ds_cb_${d}_$v.txt 2>&1 || { tail -5 gpurun_out/r3ds_cb_${d}_$v.txt; exit 1; }
    echo "short=$v $d: $(tail -2 gpurun_out/r3ds_cb_${d}_$v.txt | head -1)"
  done
done
C="--no-infer --no-cpu-baseline --no-roofline --no-sweep --no-infer-sweep --no-bf16 --exact-steps 0 --steps 10 --warmup 3"
for r in 1 2; do
  for v in 0 1; do
    MAUV_DGRAD_SHORT=$v timeout -k 10 300 python -u bench.py --dtype bf16 $C > gpurun_out/r3ds_b_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r3ds_b_${v}_$r.log; exit 1; }
    MAUV_DGRAD_SHORT=$v timeout -k 10 300 python -u bench.py $C > gpurun_out/r3ds_f_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r3ds_f_${v}_$r.log; exit 1; }
    echo "short=$v round $r: bf16 $(grep -o '"value": [0-9.]*' gpurun_out/r3ds_b_${v}_$r.log | head -1) fp32 $(grep -o '"value": [0-9.]*' gpurun_out/r3ds_f_${v}_$r.log | head -1)"
  done
done
echo done
