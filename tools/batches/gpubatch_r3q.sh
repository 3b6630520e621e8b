# RECORD ONLY: the switches / experimental libraries this script A/Bs were removed after the measurement (profiles/round3/*_ab.txt); it no longer runs against the current library
# round 3: gradient arena attached during the forward (host work off the loss-check -> backward
# critical path), and the BN backward partial pass with U rows' loads issued together
# (MAUV_BN_PUNROLL = 1 / 2 / 4): model, drop-in and BN tests; serial kernel statistics per U;
# interleaved bf16 legs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MAUV_BN_PUNROLL=4 timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "model or dropin or ddp or bn or adam or bench or kl" > gpurun_out/r3q_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r3q_tests.log | head; tail -5 gpurun_out/r3q_tests.log; exit 1; }
tail -1 gpurun_out/r3q_tests.log
for u in 1 2 4; do
  MAUV_BN_PUNROLL=$u MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3q_st16_$u -o run -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer --no-bf16 > gpurun_out/r3q_st16_$u.log 2>&1 || exit 1
done
B16="--no-cpu-baseline --no-roofline --no-sweep --no-infer --no-bf16 --exact-steps 0 --steps 8 --warmup 2 --dtype bf16"
for r in 1 2; do
  for u in 1 2 4; do
    MAUV_BN_PUNROLL=$u timeout -k 10 300 python -u bench.py $B16 > gpurun_out/r3q_b16_${u}_$r.log 2>&1 || { tail -5 gpurun_out/r3q_b16_${u}_$r.log; exit 1; }
    echo "punroll=$u round $r: bf16 $(tail -1 gpurun_out/r3q_b16_${u}_$r.log | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["value"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3q_cc16 -o run -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer --no-bf16 > gpurun_out/r3q_cc16.log 2>&1 || exit 1
echo done
