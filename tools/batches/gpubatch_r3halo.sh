# round 3: the 3x3 / stride-1 / 64 -> 64 16-bit forward through an LDS image of the input rows
# (conv_halo16.hip) — bit-identity against the implicit GEMM, per-shape forwards with
# MAUV_HALO3=0/1 (training slice and an f16 inference chunk), then interleaved A/Bs of the bf16
# step and the f16 inference leg
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_halo16_gpu.py tests/test_kernels16_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3halo_test.log 2>&1 || { tail -30 gpurun_out/r3halo_test.log; exit 1; }
tail -2 gpurun_out/r3halo_test.log
for v in 0 1; do
  MAUV_HALO3=$v timeout -k 10 300 python -u tools/conv_bench.py --dtype bf16 --fused --only fwd,dgrad --top 400 > gpurun_out/r3halo_cb_b_$v.txt 2>&1 || { tail -5 gpurun_out/r3halo_cb_b_$v.txt; exit 1; }
  MAUV_HALO3=$v timeout -k 10 300 python -u tools/conv_bench.py --dtype f16 --fused --G 10 --B 256 --only fwd --top 400 > gpurun_out/r3halo_cb_i_$v.txt 2>&1 || { tail -5 gpurun_out/r3halo_cb_i_$v.txt; exit 1; }
  echo "halo=$v bf16: $(grep "(64, 64, 3, 1, 1, 64)" gpurun_out/r3halo_cb_b_$v.txt | head -1)"
  echo "halo=$v bf16: $(grep "(64, 64, 3, 1, 1, 56)" gpurun_out/r3halo_cb_b_$v.txt | head -1)"
  echo "halo=$v bf16: $(grep "dgrad  (64, 64, 3, 1, 1, 64)" gpurun_out/r3halo_cb_b_$v.txt | head -1)"
  echo "halo=$v bf16: $(grep "dgrad  (64, 64, 3, 1, 1, 56)" gpurun_out/r3halo_cb_b_$v.txt | head -1)"
  echo "halo=$v f16 : $(grep "(64, 64, 3, 1, 1, 64)" gpurun_out/r3halo_cb_i_$v.txt | head -1)"
  echo "halo=$v f16 : $(grep "(64, 64, 3, 1, 1, 56)" gpurun_out/r3halo_cb_i_$v.txt | head -1)"
done
C="--no-cpu-baseline --no-roofline --no-sweep --no-infer-sweep --no-bf16 --exact-steps 0 --no-infer-fp32 --steps 8 --warmup 2 --dtype bf16"
for r in 1 2; do
  for v in 0 1; do
    MAUV_HALO3=$v timeout -k 10 400 python -u bench.py $C > gpurun_out/r3halo_b_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r3halo_b_${v}_$r.log; exit 1; }
    echo "halo=$v round $r: $(python3 -c "import json;d=json.loads(open('gpurun_out/r3halo_b_${v}_$r.log').read().strip().splitlines()[-1]);print('bf16', d['value'], 'infer', d['inference']['value'])")"
  done
done
echo done
