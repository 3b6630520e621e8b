# RECORD ONLY: the switches / experimental libraries this script A/Bs were removed after the measurement (profiles/round3/*_ab.txt); it no longer runs against the current library
# round 3: BN finalize geometry, experimental libraries (MAUV_LIB): v1 = backward partial blocks
# capped at 256 per group (was 1024: the finalize walks 4x fewer partials), v2 = forward statistics
# segments of 128 partials (was 512: 4x more finalize blocks, shorter chains), v3 = both.
# BN / model tests per library, serial bf16 kernel statistics, interleaved bf16 + f16 inference legs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=multimodal-auv_amd/mauv
for v in v1 v2 v3; do
  MAUV_LIB=$P/libmauv_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernels16_gpu.py tests/test_bwd_fusion_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread -k "bn or model or train" > gpurun_out/r3r_tests_$v.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r3r_tests_$v.log | head; tail -5 gpurun_out/r3r_tests_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/r3r_tests_$v.log)"
done
for v in base v1 v2 v3; do
  L=$P/libmauv_hip.so; [ $v != base ] && L=$P/libmauv_hip_$v.so
  MAUV_LIB=$L MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3r_st16_$v -o run -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer --no-bf16 > gpurun_out/r3r_st16_$v.log 2>&1 || exit 1
done
C="--no-cpu-baseline --no-roofline --no-sweep --no-infer-sweep --no-bf16 --exact-steps 0 --no-infer-fp32 --steps 8 --warmup 2 --dtype bf16"
for r in 1 2; do
  for v in base v1 v2 v3; do
    L=$P/libmauv_hip.so; [ $v != base ] && L=$P/libmauv_hip_$v.so
    MAUV_LIB=$L timeout -k 10 400 python -u bench.py $C > gpurun_out/r3r_b_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r3r_b_${v}_$r.log; exit 1; }
    echo "$v round $r: $(python3 -c "import json;d=json.loads(open('gpurun_out/r3r_b_${v}_$r.log').read().strip().splitlines()[-1]);print('bf16', d['value'], 'infer', d['inference']['value'])")"
  done
done
echo done
