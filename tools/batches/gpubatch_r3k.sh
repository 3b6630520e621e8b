# round 3: reparam_bwd — one thread per (sample, element) slab reduction, up to 8 samples' images per parameter pass — kernel tests, then an
# interleaved same-box A/B against the previous library (MAUV_LIB) of the bf16 and fp32 steps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py::test_reparam_and_kl tests/test_kernels_gpu.py::test_reparam_bwd_sample_batches tests/test_kernels16_gpu.py tests/test_model_gpu.py::test_multimodal_train_step_parity tests/test_model_gpu.py::test_exact_rho_gradient_mode tests/test_model_gpu.py::test_mc_batched_equals_sequential -v -s --timeout 200 --timeout-method thread > gpurun_out/r3k_test.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/r3k_test.log | tail -12
[ $rc -eq 0 ] || { echo "tests rc=$rc: stop"; exit $rc; }
C="--no-infer --no-cpu-baseline --no-roofline --no-sweep --no-infer-sweep --no-bf16 --exact-steps 0 --steps 10 --warmup 3"
P=multimodal-auv_amd/mauv
for r in 1 2 3; do
  for v in prev new; do
    L=$P/libmauv_hip.so; [ $v = prev ] && L=$P/libmauv_hip_prev.so
    MAUV_LIB=$L timeout -k 10 300 python -u bench.py --dtype bf16 $C > gpurun_out/r3k_b_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r3k_b_${v}_$r.log; exit 1; }
    MAUV_LIB=$L timeout -k 10 300 python -u bench.py $C > gpurun_out/r3k_f_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r3k_f_${v}_$r.log; exit 1; }
    echo "$v round $r: bf16 $(grep -o '"value": [0-9.]*' gpurun_out/r3k_b_${v}_$r.log | head -1) fp32 $(grep -o '"value": [0-9.]*' gpurun_out/r3k_f_${v}_$r.log | head -1)"
  done
done
for v in prev new; do
  L=$P/libmauv_hip.so; [ $v = prev ] && L=$P/libmauv_hip_prev.so
  MAUV_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3k_prof_$v -o run -- python3 bench.py --dtype bf16 --no-infer --no-cpu-baseline --no-roofline --no-sweep --no-infer-sweep --no-bf16 --exact-steps 0 --steps 3 --warmup 1 > gpurun_out/r3k_prof_$v.log 2>&1 || { tail -5 gpurun_out/r3k_prof_$v.log; exit 1; }
done
echo done
