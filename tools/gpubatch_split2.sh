# split-fp32: accuracy per mode, per-shape timing for the tile-depth / accumulator variants,
# and SQ counters of one 3x3 shape (split vs exact)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/f32_math_diag.py > gpurun_out/diag_acc.log 2>&1 || exit 1
for v in "split 16" "split 32" "split1 16" "split1 32"; do
  set -- $v
  MAUV_F32_MATH=$1 MAUV_SPLIT_BK=$2 timeout -k 10 300 python -u tools/conv_bench.py --reps 3 --top 40 > gpurun_out/cb_$1_$2.log 2>&1 || exit 1
done
SHAPE="--trunks opt --shape 128,128,3,1,1,32 --reps 3"
for m in split exact; do
  MAUV_F32_MATH=$m timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_$m -o run -- python3 tools/conv_bench.py $SHAPE > gpurun_out/pmc_$m.log 2>&1 || exit 1
  MAUV_F32_MATH=$m timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc2_$m -o run -- python3 tools/conv_bench.py $SHAPE > gpurun_out/pmc2_$m.log 2>&1 || exit 1
done
echo done
