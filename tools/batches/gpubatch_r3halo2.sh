# round 3: conv_halo16 with every tap's weight slice fetched up front (no global loads in the tap
# loop) against the previous library (MAUV_LIB=libmauv_hip_prev.so): halo tests, per-shape
# timings of the 3x3 64->64 forwards / data gradients, interleaved bench legs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=multimodal-auv_amd/mauv
timeout -k 10 300 python -u -m pytest tests/test_halo16_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3h2_test.log 2>&1 || { tail -30 gpurun_out/r3h2_test.log; exit 1; }
tail -1 gpurun_out/r3h2_test.log
for v in prev new; do
  L=$P/libmauv_hip.so; [ $v = prev ] && L=$P/libmauv_hip_prev.so
  MAUV_LIB=$L timeout -k 10 300 python -u tools/conv_bench.py --dtype bf16 --fused --only fwd,dgrad --top 400 --shape 64,64,3,1,1,64 --trunks bathy --reps 20 > gpurun_out/r3h2_cb64_$v.txt 2>&1 || { tail -5 gpurun_out/r3h2_cb64_$v.txt; exit 1; }
  MAUV_LIB=$L timeout -k 10 300 python -u tools/conv_bench.py --dtype bf16 --fused --only fwd,dgrad --top 400 --shape 64,64,3,1,1,56 --trunks opt --reps 20 > gpurun_out/r3h2_cb56_$v.txt 2>&1 || { tail -5 gpurun_out/r3h2_cb56_$v.txt; exit 1; }
  MAUV_LIB=$L timeout -k 10 300 python -u tools/conv_bench.py --dtype f16 --fused --G 10 --B 256 --only fwd --shape 64,64,3,1,1,64 --trunks bathy --reps 5 > gpurun_out/r3h2_cbi_$v.txt 2>&1 || { tail -5 gpurun_out/r3h2_cbi_$v.txt; exit 1; }
  echo "$v: $(grep -h "shape" gpurun_out/r3h2_cb64_$v.txt gpurun_out/r3h2_cb56_$v.txt gpurun_out/r3h2_cbi_$v.txt | awk '{print $3, $4,$5,$6,$7,$8,$9, $10}' | tr '\n' '|')"
done
C="--no-cpu-baseline --no-roofline --no-sweep --no-infer-sweep --no-bf16 --exact-steps 0 --no-infer-fp32 --steps 8 --warmup 2 --dtype bf16"
for r in 1 2; do
  for v in prev new; do
    L=$P/libmauv_hip.so; [ $v = prev ] && L=$P/libmauv_hip_prev.so
    MAUV_LIB=$L timeout -k 10 400 python -u bench.py $C > gpurun_out/r3h2_b_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r3h2_b_${v}_$r.log; exit 1; }
    echo "$v round $r: $(python3 -c "import json;d=json.loads(open('gpurun_out/r3h2_b_${v}_$r.log').read().strip().splitlines()[-1]);print('bf16', d['value'], 'infer', d['inference']['value'])")"
  done
done
echo done
