# round 3: BN-backward partials from the 16-bit data-gradient epilogue — kernel test, 16-bit
# parity tests, then an interleaved same-box A/B of the bf16 step (MAUV_DGRAD_BN_EPI=0/1)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels16_gpu.py -k "bn_partials or fwd_dgrad_wgrad" tests/test_parity16_gpu.py::test_train_step16_grads_vs_torch_autocast tests/test_model_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r3g_test.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert|whole-gradient|median" gpurun_out/r3g_test.log | tail -40
[ $rc -eq 0 ] || { echo "tests rc=$rc: stop"; exit $rc; }
B="python -u bench.py --dtype bf16 --no-infer --no-cpu-baseline --no-roofline --no-sweep --no-infer-sweep --no-bf16 --exact-steps 0 --steps 10 --warmup 3"
for r in 1 2; do
  for v in 0 1; do
    MAUV_DGRAD_BN_EPI=$v timeout -k 10 300 $B > gpurun_out/r3g_ab_${v}_${r}.log 2> gpurun_out/r3g_ab_${v}_${r}.err || { tail -5 gpurun_out/r3g_ab_${v}_${r}.err; exit 1; }
    echo "epi=$v round $r: $(grep -o '"value": [0-9.]*' gpurun_out/r3g_ab_${v}_${r}.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3g_ab_${v}_${r}.log | head -1)"
  done
done
echo done
