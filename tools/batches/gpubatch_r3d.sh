# round 3: DMA bit-identity + class-agreement tests, interleaved per-shape A/B of the LDS-DMA
# kernels, the default bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels16_gpu.py -k dma tests/test_parity16_gpu.py tests/test_configs4_gpu.py -v -s --timeout 400 --timeout-method thread > gpurun_out/r3d_new.log 2>&1
rc=$?
grep -E "PASS|FAIL|classes|S=|Error" gpurun_out/r3d_new.log | tail -40
case $rc in 0|1) ;; *) echo "new tests rc=$rc: stop"; exit $rc;; esac
timeout -k 10 400 python -u tools/dma_ab.py --dtype bf16 > gpurun_out/r3d_ab_bf16.log 2>&1 || exit 1
grep TOTAL gpurun_out/r3d_ab_bf16.log
timeout -k 10 700 python -u bench.py > gpurun_out/r3d_bench.log 2> gpurun_out/r3d_bench.err || { tail -20 gpurun_out/r3d_bench.err; exit 1; }
tail -c 3500 gpurun_out/r3d_bench.log
echo done
