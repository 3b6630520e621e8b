# One gpurun call that produces a round's evidence on one box, in order:
#   the full GPU suite (-rP: the parity tests' printed deviations are kept) and smoke(),
#   PMC traffic of both conv families on this library (copied where bench.py reads it),
#   the default bench line, serial kernel statistics of the steady fp32 and bf16 steps
#   (tools/steady_stats.py: setup and the warm-up step excluded), and
#   kernel statistics of the f16 inference leg.
# usage (from the repo root, on the box):  bash tools/gpu_evidence.sh TAG [all|tests|rest]
#   (a gpurun call is capped at 20 minutes: run "tests" and "rest" as two calls)
#   outputs under gpurun_out/TAG_*; the traffic summaries as profiles/TAG[_bf16]_conv_traffic.json
set -o pipefail
TAG=${1:?tag}
mkdir -p gpurun_out
export TMPDIR=/tmp
PART=${2:-all}
if [ "$PART" != "rest" ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/${TAG}_tests.log | head; tail -5 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
  tail -1 gpurun_out/${TAG}_smoke.log
fi
[ "$PART" = "tests" ] && exit 0
B32="bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline --no-sweep"
B16="bench.py --dtype bf16 --steps 1 --warmup 0 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline --no-sweep"
for pass in "f32 FETCH_SIZE fetch $B32" "f32 WRITE_SIZE write $B32" "b16 FETCH_SIZE fetch $B16" "b16 WRITE_SIZE write $B16"; do
  set -- $pass
  fam=$1; ctr=$2; kind=$3; shift 3
  MAUV_TRUNK_STREAMS=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d gpurun_out/${TAG}_pmc_${fam}_${kind} -o run -- python3 "$@" > gpurun_out/${TAG}_pmc_${fam}_${kind}.log 2>&1 || exit 1
done
python3 tools/pmc_traffic.py gpurun_out/${TAG}_pmc_f32_fetch gpurun_out/${TAG}_pmc_f32_write gpurun_out/${TAG}_conv_traffic.json > gpurun_out/${TAG}_pmc_f32_summary.txt || exit 1
python3 tools/pmc_traffic.py gpurun_out/${TAG}_pmc_b16_fetch gpurun_out/${TAG}_pmc_b16_write gpurun_out/${TAG}_bf16_conv_traffic.json > gpurun_out/${TAG}_pmc_b16_summary.txt || exit 1
cp gpurun_out/${TAG}_conv_traffic.json gpurun_out/${TAG}_bf16_conv_traffic.json profiles/ || exit 1
timeout -k 10 1200 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_bench.json
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print(d['value'], d['bf16_train']['value'], d['inference']['value'], d['roofline']['frac'], d['roofline']['traffic_matches_library'], d['bf16_train']['roofline']['frac'], d['bf16_train']['roofline']['traffic_matches_library'])"
C="--no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer --no-bf16"
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_st32 -o run -- python3 bench.py --steps 2 --warmup 1 $C > gpurun_out/${TAG}_st32.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_st16 -o run -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 $C > gpurun_out/${TAG}_st16.log 2>&1 || exit 1
# per-kernel statistics of the steady steps only (setup and the warm-up step excluded)
python3 tools/steady_stats.py gpurun_out/${TAG}_st32 gpurun_out/${TAG}_train_step_kernel_stats_steady.csv || exit 1
python3 tools/steady_stats.py gpurun_out/${TAG}_st16 gpurun_out/${TAG}_bf16_train_step_kernel_stats_steady.csv || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_inf -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer-sweep --no-bf16 --no-infer-fp32 > gpurun_out/${TAG}_inf.log 2>&1 || exit 1
echo done
