# round 3: 16-bit data gradients through the short-K kernels with the BN-partials epilogue
# compiled out (69-71 VGPRs, no scratch; the round-3 A/B of gpubatch_r3ds.sh spilled 152-192 B
# per lane) — kernel parity, per-shape data-gradient timings with MAUV_DGRAD_SHORT=0/1, then an
# interleaved same-box A/B of the bf16 step and the f16 inference leg
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_kernels16_gpu.py tests/test_bwd_fusion_gpu.py tests/test_kernels_gpu.py::test_dgrad_accumulate_into_dx -x -q --timeout 200 --timeout-method thread > gpurun_out/r3ds2_test.log 2>&1 || { tail -30 gpurun_out/r3ds2_test.log; exit 1; }
tail -2 gpurun_out/r3ds2_test.log
for v in 0 1; do
  MAUV_DGRAD_SHORT=$v timeout -k 10 300 python -u tools/conv_bench.py --dtype bf16 --only dgrad --top 400 > gpurun_out/r3ds2_cb_$v.txt 2>&1 || { tail -5 gpurun_out/r3ds2_cb_$v.txt; exit 1; }
  echo "short=$v: $(tail -2 gpurun_out/r3ds2_cb_$v.txt | head -1)"
done
C="--no-infer --no-cpu-baseline --no-roofline --no-sweep --no-infer-sweep --no-bf16 --exact-steps 0 --steps 10 --warmup 3"
for r in 1 2 3; do
  for v in 0 1; do
    MAUV_DGRAD_SHORT=$v timeout -k 10 300 python -u bench.py --dtype bf16 $C > gpurun_out/r3ds2_b_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r3ds2_b_${v}_$r.log; exit 1; }
    echo "short=$v round $r: bf16 $(grep -o '"value": [0-9.]*' gpurun_out/r3ds2_b_${v}_$r.log | head -1)"
  done
done
echo done
