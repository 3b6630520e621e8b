#!/bin/bash
# round-5 GPU call 7: 16-bit BN-backward partials from the data-gradient epilogue (engine
# BWD_PARTIALS_16) — kernel / model tests, same-box A/B of the bf16 step, serial kernel
# statistics of a bf16 step with the switch off and on (BN share)
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c7; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 "$@" > $O/$n.log 2>&1; local r=$?; echo "$n rc=$r"; [ $r -eq 0 ]; }
run tests 600 python -u -m pytest -v -rP --timeout 300 --timeout-method thread tests/test_bwd_fusion_gpu.py || exit 1
run ab 600 python -u tools/fold_ab.py --train --dtype bf16 --flag BWD_PARTIALS_16 --rounds 4 --steps 10 || exit 1
C="--no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer --no-bf16"
for v in 0 1; do
  MAUV_BWD_PARTIALS_16=$v MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st16_$v -o run -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 $C > $O/st16_$v.log 2>&1 || { echo "st16_$v failed"; exit 1; }
done
echo done
