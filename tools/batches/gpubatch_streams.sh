# RECORD ONLY: the switch MAUV_SIDE_WGRAD and the variant it selected were measured (DESIGN.md cites the result)
# and removed from the code; this script no longer reproduces that A/B.
# concurrent trunk streams: model parity + A/B bench (fp32, bf16, inference)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_model_gpu.py tests/test_model16_gpu.py > gpurun_out/t_tests.log 2>&1 || { tail -30 gpurun_out/t_tests.log; exit 1; }
tail -n 1 gpurun_out/t_tests.log
for E in 0 1 0 1; do export MAUV_SIDE_WGRAD=$E
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline > gpurun_out/sw_$E.log 2>&1 || exit 1
python3 - gpurun_out/sw_$E.log $E <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("E=",sys.argv[2],"fp32",d["value"],"bf16",d["bf16_train"]["value"],"inf",d["inference"]["value"])
PY
done
echo done
