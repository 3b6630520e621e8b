# PMC on one memory-bound 16-bit shape: 1x1 64->256 over 64x64, G=2, B=256, f16, fused (XBN)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SHAPE="--dtype f16 --trunks opt --shape 64,256,1,1,0,64 --reps 3 --only fwd --B 256 --G 2 --fused"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/ms_a -o run -- python3 tools/conv_bench.py $SHAPE > gpurun_out/ms_a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/ms_b -o run -- python3 tools/conv_bench.py $SHAPE > gpurun_out/ms_b.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/ms_c -o run -- python3 tools/conv_bench.py $SHAPE > gpurun_out/ms_c.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/ms_d -o run -- python3 tools/conv_bench.py $SHAPE > gpurun_out/ms_d.log 2>&1 || exit 1
grep -h "shape" gpurun_out/ms_a.log | head -2
echo done
