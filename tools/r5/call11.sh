#!/bin/bash
# round-5 GPU call 11: whole-step A/Bs of conv_expand16's default routing (bf16 step, f16 inference)
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c11; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 "$@" > $O/$n.log 2>&1; local r=$?; echo "$n rc=$r"; [ $r -eq 0 ]; }
run infer 600 python -u tools/fold_ab.py --flag expand16 --rounds 4 || exit 1
run train 500 python -u tools/fold_ab.py --train --dtype bf16 --flag expand16 --rounds 4 --steps 10 || exit 1
echo done
