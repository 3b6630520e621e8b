# round 3: new tests (+ the LDS-DMA 16-bit kernels' bit-identity), per-shape A/B of the LDS-DMA
# kernels against the pipelined ones (bf16, training slice G=5 B=64), the default bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels16_gpu.py tests/test_kl_gpu.py tests/test_resize.py tests/test_parity16_gpu.py tests/test_configs4_gpu.py -v -s --timeout 400 --timeout-method thread > gpurun_out/r3c_new.log 2>&1
rc=$?
grep -E "PASS|FAIL|cos vs|dlogit|classes|KL |S=|Error" gpurun_out/r3c_new.log | tail -60
case $rc in 0|1) ;; *) echo "new tests rc=$rc: stop"; exit $rc;; esac
for d in 1 0; do
  timeout -k 10 300 python -u tools/conv_bench.py --dtype bf16 --only fwd,dgrad --dma $d --top 12 > gpurun_out/r3c_cb_dma$d.log 2>&1 || exit 1
  echo "== dma=$d"; grep -E "TOTAL|rsck" gpurun_out/r3c_cb_dma$d.log | head -8
done
timeout -k 10 700 python -u bench.py > gpurun_out/r3c_bench.log 2>&1 || { tail -20 gpurun_out/r3c_bench.log; exit 1; }
tail -c 3000 gpurun_out/r3c_bench.log
echo done
