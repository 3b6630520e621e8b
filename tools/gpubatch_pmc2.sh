set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SHAPE="--trunks opt --shape 128,128,3,1,1,32 --reps 3 --only fwd"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/p5a -o run -- python3 tools/conv_bench.py $SHAPE > gpurun_out/p5a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/p5b -o run -- python3 tools/conv_bench.py $SHAPE > gpurun_out/p5b.log 2>&1 || exit 1
echo done
