# pipelined split-fp32 kernel: parity (kernels, fused-BN conv paths, model), accuracy per mode,
# per-shape timing (split = 2 accumulators, split1 = 1), short training bench
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_f32_math_gpu.py tests/test_kernels_gpu.py > gpurun_out/s3_kern.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/f32_math_diag.py exact,split,split1 > gpurun_out/s3_diag.log 2>&1 || exit 1
for m in split split1; do
  MAUV_F32_MATH=$m timeout -k 10 300 python -u tools/conv_bench.py --reps 3 --top 30 > gpurun_out/s3_cb_$m.log 2>&1 || exit 1
  MAUV_F32_MATH=$m timeout -k 10 300 python -u tools/conv_bench.py --reps 3 --top 10 --fused > gpurun_out/s3_cbf_$m.log 2>&1 || exit 1
done
timeout -k 10 600 $T tests/test_model_gpu.py > gpurun_out/s3_model.log 2>&1 || exit 1
for m in split split1; do
  MAUV_F32_MATH=$m timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --steps 4 --warmup 1 > gpurun_out/s3_bench_$m.log 2>&1 || exit 1
done
echo done
