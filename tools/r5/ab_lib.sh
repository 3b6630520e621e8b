#!/bin/bash
# same-box A/B of two libraries on bench legs: tools/r5/ab_lib.sh OUTDIR ROUNDS BASE_LIB -- bench args
# (interleaved: base, new, new, base, ...); prints one summary line per run
O=$1; R=$2; BASE=$3; shift 4
mkdir -p $O
for i in $(seq 1 $R); do
  if [ $((i % 2)) -eq 1 ]; then order="base new"; else order="new base"; fi
  for arm in $order; do
    if [ $arm = base ]; then L=$BASE; else L=multimodal-auv_amd/mauv/libmauv_hip.so; fi
    MAUV_LIB=$L timeout -k 10 400 python -u bench.py "$@" > $O/${arm}_$i.log 2>&1 || { echo "$arm $i failed rc=$?"; tail -5 $O/${arm}_$i.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('$O/${arm}_$i.log').read().strip().splitlines()[-1])
b=d.get('bf16_train') or {}
i_=d.get('inference') or {}
print('$arm', $i, 'fp32', d['value'], 'bf16', b.get('value'), 'infer', i_.get('value'))"
  done
done
