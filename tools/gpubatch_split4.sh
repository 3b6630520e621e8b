# pipelined split kernel: SQ counters on one 3x3 shape, bf16 kernel timing for reference, bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SHAPE="--trunks opt --shape 128,128,3,1,1,32 --reps 3"
for only in fwd wgrad; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/p4a_$only -o run -- python3 tools/conv_bench.py $SHAPE --only $only > gpurun_out/p4a_$only.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/p4b_$only -o run -- python3 tools/conv_bench.py $SHAPE --only $only > gpurun_out/p4b_$only.log 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/conv_bench.py --reps 3 --top 10 --dtype bf16 > gpurun_out/s4_cb_bf16.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-infer --no-bf16 --steps 4 --warmup 1 > gpurun_out/s4_bench.log 2>&1 || exit 1
echo done
