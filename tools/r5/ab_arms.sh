#!/bin/bash
# same-box interleaved A/B/C of bench legs: tools/r5/ab_arms.sh OUTDIR ROUNDS "name|ENV=.. ENV2=.." ... -- bench args
# each arm is a label and env assignments (e.g. "base|MAUV_LIB=multimodal-auv_amd/mauv/libmauv_hip_base.so")
O=$1; R=$2; shift 2
ARMS=()
while [ "$1" != "--" ]; do ARMS+=("$1"); shift; done
shift
mkdir -p $O
n=${#ARMS[@]}
for i in $(seq 1 $R); do
  for j in $(seq 0 $((n - 1))); do
    k=$(( (j + i - 1) % n ))
    spec=${ARMS[$k]}; name=${spec%%|*}; envs=${spec#*|}
    env $envs timeout -k 10 400 python -u bench.py "$@" > $O/${name}_$i.log 2>&1 || { echo "$name $i failed"; tail -5 $O/${name}_$i.log; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/${name}_$i.log').read().strip().splitlines()[-1])
b=d.get('bf16_train') or {}
f=d.get('inference') or {}
print('$name', $i, 'fp32', d['value'], 'bf16', b.get('value'), 'infer', f.get('value'), flush=True)"
  done
done
