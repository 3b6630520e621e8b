# branch-free conv loaders (sel_off / bitwise validity / WGRAD pixel carry with 32-bit magic
# divisions, uniform tile indices in SGPRs) against the previous library (tools/ab/libmauv_prev.so,
# built from the commit before): conv kernel parity, conv totals, training + inference A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
PREV=$PWD/tools/ab/libmauv_prev.so
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernels16_gpu.py tests/test_f32_math_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s3r_tests.log 2>&1 || { tail -30 gpurun_out/s3r_tests.log; exit 1; }
tail -1 gpurun_out/s3r_tests.log
for lib in new prev; do
  L=""; [ $lib = prev ] && L=$PREV
  for dt in fp32 bf16; do
    MAUV_LIB=${L:-$PWD/multimodal-auv_amd/mauv/libmauv_hip.so} timeout -k 10 200 python -u tools/conv_bench.py --dtype $dt --fused --top 0 > gpurun_out/s3r_cb_${dt}_$lib.txt 2>&1 || exit 1
    echo "$lib $dt"; grep TOTAL gpurun_out/s3r_cb_${dt}_$lib.txt
  done
done
B="--no-cpu-baseline --exact-steps 0 --no-roofline"
for lib in prev new prev new; do
  L=$PWD/multimodal-auv_amd/mauv/libmauv_hip.so; [ $lib = prev ] && L=$PREV
  MAUV_LIB=$L timeout -k 10 300 python -u bench.py $B --no-infer > gpurun_out/s3r_tr.log 2>&1 || { tail -5 gpurun_out/s3r_tr.log; exit 1; }
  echo "$lib train"; tail -1 gpurun_out/s3r_tr.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['bf16_train']['value'])"
done
for lib in prev new; do
  L=$PWD/multimodal-auv_amd/mauv/libmauv_hip.so; [ $lib = prev ] && L=$PREV
  MAUV_LIB=$L timeout -k 10 300 python -u bench.py $B --no-bf16 --no-infer-fp32 --steps 1 --warmup 1 > gpurun_out/s3r_inf.log 2>&1 || { tail -5 gpurun_out/s3r_inf.log; exit 1; }
  echo "$lib infer"; tail -1 gpurun_out/s3r_inf.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['inference']['value'])"
done
