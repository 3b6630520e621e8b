# round 3 (resumed session): the full GPU suite and smoke() on the tree after the conv_halo16
# weight-prefetch change, plus per-shape bf16 timings of the stems and the 3x3 64->64 weight gradient
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3l_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r3l_tests.log | head; tail -5 gpurun_out/r3l_tests.log; exit 1; }
tail -1 gpurun_out/r3l_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3l_smoke.log 2>&1 || { tail -20 gpurun_out/r3l_smoke.log; exit 1; }
tail -1 gpurun_out/r3l_smoke.log
timeout -k 10 300 python -u tools/conv_bench.py --dtype bf16 --fused --top 40 --reps 10 > gpurun_out/r3l_convbench_bf16.txt 2>&1 || { tail -5 gpurun_out/r3l_convbench_bf16.txt; exit 1; }
echo done
