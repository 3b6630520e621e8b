# 16-bit conv: full per-shape listing + SQ counters on one 3x3 shape (fwd)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/conv_bench.py --dtype bf16 --top 200 --trunks bathy > gpurun_out/q16_all.log 2>&1 || exit 1
SHAPE="--dtype bf16 --trunks opt --shape 256,256,3,1,1,16 --reps 3 --only fwd"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/q16a -o run -- python3 tools/conv_bench.py $SHAPE > gpurun_out/q16a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_MFMA --output-format csv -d gpurun_out/q16b -o run -- python3 tools/conv_bench.py $SHAPE > gpurun_out/q16b.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/q16c -o run -- python3 tools/conv_bench.py $SHAPE > gpurun_out/q16c.log 2>&1 || exit 1
echo done
