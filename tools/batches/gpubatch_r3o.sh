# RECORD ONLY: the switches / experimental libraries this script A/Bs were removed after the measurement (profiles/round3/*_ab.txt); it no longer runs against the current library
# round 3: block order of the BN row passes (MAUV_BN_REV bits: 1 = backward partial pass reversed,
# 2 = backward apply reversed, 4 = forward apply reversed) — a pass that walks its tensors in the
# opposite order of the pass before starts on the rows the memory-side cache still holds.
# BN tests under the reversed orders, interleaved bf16 legs, serial kernel statistics per arm.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MAUV_BN_REV=7 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernels16_gpu.py tests/test_bwd_fusion_gpu.py -x -q --timeout 200 --timeout-method thread -k "bn" > gpurun_out/r3o_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r3o_tests.log | head; tail -5 gpurun_out/r3o_tests.log; exit 1; }
tail -1 gpurun_out/r3o_tests.log
B16="--no-cpu-baseline --no-roofline --no-sweep --no-infer --no-bf16 --exact-steps 0 --steps 8 --warmup 2 --dtype bf16"
for r in 1 2; do
  for m in 0 1 5 2 6; do
    MAUV_BN_REV=$m timeout -k 10 300 python -u bench.py $B16 > gpurun_out/r3o_b16_${m}_$r.log 2>&1 || { tail -5 gpurun_out/r3o_b16_${m}_$r.log; exit 1; }
    echo "rev=$m round $r: bf16 $(tail -1 gpurun_out/r3o_b16_${m}_$r.log | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["value"])')"
  done
done
for m in 0 1 5; do
  MAUV_BN_REV=$m MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3o_st16_$m -o run -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer --no-bf16 > gpurun_out/r3o_st16_$m.log 2>&1 || exit 1
done
echo done
