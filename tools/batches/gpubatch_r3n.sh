# round 3: 16-byte reparam_bwd (reparam_bwd4) + block-form sampling (MAUV_REPARAM_BWD4 = MAUV_SAMPLE_BLK = 1, defaults)
# kernel (=0), and the 8-channel max-pool backward: kernel tests, the model-gradient tests,
# interleaved bf16 / fp32 training legs, one serial bf16 step's kernel statistics
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernels16_gpu.py -x -q --timeout 200 --timeout-method thread -k "reparam or pool or adam" > gpurun_out/r3n_ktests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/r3n_ktests.log | head -20; tail -5 gpurun_out/r3n_ktests.log; exit 1; }
tail -1 gpurun_out/r3n_ktests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "model or dropin or grad or train" > gpurun_out/r3n_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r3n_tests.log | head; tail -5 gpurun_out/r3n_tests.log; exit 1; }
tail -1 gpurun_out/r3n_tests.log
B16="--no-cpu-baseline --no-roofline --no-sweep --no-infer --no-bf16 --exact-steps 0 --steps 8 --warmup 2 --dtype bf16"
B32="--no-cpu-baseline --no-roofline --no-sweep --no-infer --no-bf16 --exact-steps 0 --steps 6 --warmup 2"
for r in 1 2; do
  for m in 0 1; do
    MAUV_REPARAM_BWD4=$m MAUV_SAMPLE_BLK=$m timeout -k 10 300 python -u bench.py $B16 > gpurun_out/r3n_b16_${m}_$r.log 2>&1 || { tail -5 gpurun_out/r3n_b16_${m}_$r.log; exit 1; }
    MAUV_REPARAM_BWD4=$m MAUV_SAMPLE_BLK=$m timeout -k 10 300 python -u bench.py $B32 > gpurun_out/r3n_b32_${m}_$r.log 2>&1 || { tail -5 gpurun_out/r3n_b32_${m}_$r.log; exit 1; }
    echo "bwd4=$m round $r: bf16 $(tail -1 gpurun_out/r3n_b16_${m}_$r.log | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["value"])') fp32 $(tail -1 gpurun_out/r3n_b32_${m}_$r.log | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["value"])')"
  done
done
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3n_st16 -o run -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer --no-bf16 > gpurun_out/r3n_st16.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 python -u -m cProfile -o gpurun_out/r3n_host.prof bench.py --dtype bf16 --steps 6 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer --no-bf16 > gpurun_out/r3n_host.log 2>&1 || exit 1
python3 -c "import pstats; pstats.Stats('gpurun_out/r3n_host.prof').sort_stats('tottime').print_stats(45)" > gpurun_out/r3n_host_tottime.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3n_cc16 -o run -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer --no-bf16 > gpurun_out/r3n_cc16.log 2>&1 || exit 1
echo done
