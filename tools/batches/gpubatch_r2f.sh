# round-2 evidence, part F (branch-free conv loaders, final state): PMC traffic of both conv families (separate FETCH_SIZE / WRITE_SIZE
# passes, trunks serial), the default bench line (reads that traffic), and rocprofv3 kernel
# statistics of a serial fp32 step, a serial bf16 step and one f16 inference batch
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r2f_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r2f_tests.log | head; tail -5 gpurun_out/r2f_tests.log; exit 1; }
tail -1 gpurun_out/r2f_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2f_smoke.log 2>&1 || { tail -20 gpurun_out/r2f_smoke.log; exit 1; }
tail -1 gpurun_out/r2f_smoke.log
B32="bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline"
B16="bench.py --dtype bf16 --steps 1 --warmup 0 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline"
MAUV_TRUNK_STREAMS=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/f_pmc32f -o run -- python3 $B32 > gpurun_out/f_pmc32f.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/f_pmc32w -o run -- python3 $B32 > gpurun_out/f_pmc32w.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/f_pmc16f -o run -- python3 $B16 > gpurun_out/f_pmc16f.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/f_pmc16w -o run -- python3 $B16 > gpurun_out/f_pmc16w.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/f_pmc32f gpurun_out/f_pmc32w gpurun_out/round2f_conv_traffic.json conv_f32 > gpurun_out/f_pmc32.txt || exit 1
python3 tools/pmc_traffic.py gpurun_out/f_pmc16f gpurun_out/f_pmc16w gpurun_out/round2f_bf16_conv_traffic.json conv_h16 > gpurun_out/f_pmc16.txt || exit 1
cp gpurun_out/round2f_conv_traffic.json gpurun_out/round2f_bf16_conv_traffic.json profiles/
head -3 gpurun_out/f_pmc32.txt gpurun_out/f_pmc16.txt
timeout -k 10 600 python -u bench.py > gpurun_out/round2f_bench.log 2>&1 || { tail -20 gpurun_out/round2f_bench.log; exit 1; }
tail -1 gpurun_out/round2f_bench.log > gpurun_out/round2f_bench.json
C="--no-cpu-baseline --exact-steps 0 --no-roofline"
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f_st32 -o run -- python3 bench.py --steps 2 --warmup 1 $C --no-infer --no-bf16 > gpurun_out/f_st32.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f_st16 -o run -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 $C --no-infer --no-bf16 > gpurun_out/f_st16.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f_stinf -o run -- python3 bench.py --steps 1 --warmup 0 $C --no-bf16 --no-infer-fp32 > gpurun_out/f_stinf.log 2>&1 || exit 1
echo done
bash tools/batches/gpubatch_s3traffic.sh > gpurun_out/f_shape_traffic.txt 2>&1 || exit 1
grep TOTAL gpurun_out/f_shape_traffic.txt
