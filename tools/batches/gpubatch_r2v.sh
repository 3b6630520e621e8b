# f16 lazy-BN staging without the per-word asm barrier (new lib) vs ab/lib_old.so; MC chunk sweep
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels16_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r2v_tests.log 2>&1 || { tail -30 gpurun_out/r2v_tests.log; exit 1; }
tail -1 gpurun_out/r2v_tests.log
for L in new old new old; do
  if [ $L = old ]; then export MAUV_LIB=$PWD/ab/lib_old.so; else unset MAUV_LIB; fi
  timeout -k 10 200 python -u tools/conv_bench.py --dtype f16 --G 20 --B 256 --only fwd --fused --top 3 > gpurun_out/r2v_$L.log 2>&1 || exit 1
  echo $L $(grep "TOTAL fwd" gpurun_out/r2v_$L.log)
done
unset MAUV_LIB
timeout -k 10 500 python -u tools/diag_chunk.py > gpurun_out/r2u.log 2>&1 || { tail -20 gpurun_out/r2u.log; exit 1; }
cat gpurun_out/r2u.log
