# RECORD ONLY: the switch MAUV_SIDE_WGRAD and the variant it selected were measured (DESIGN.md cites the result)
# and removed from the code; this script no longer reproduces that A/B.
# BN backward partial rows-per-thread with the ReLU masks (8/16/32), and the side wgrad stream
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "16 0" "8 0" "32 0" "16 1" "16 0" "8 0" "32 0" "16 1"; do
set -- $cfg
MAUV_BN_PARTIAL_RPT=$1 MAUV_SIDE_WGRAD=$2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline --no-infer > gpurun_out/r2_b.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/r2_b.log').read().strip().splitlines()[-1]);print('partial=$1 side=$2', d['value'], d['bf16_train']['value'])"
done
echo done
