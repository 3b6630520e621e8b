# round 2 PMC: HBM traffic of one fp32 and one bf16 training step (FETCH_SIZE / WRITE_SIZE in
# separate passes, trunks serial), then SQ counters on one representative 3x3 shape per kernel
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export MAUV_TRUNK_STREAMS=0
B32="bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline"
B16="bench.py --dtype bf16 --steps 1 --warmup 0 --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --no-roofline"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f32_fetch -o run -- python3 $B32 > gpurun_out/pmc_f32_fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_f32_write -o run -- python3 $B32 > gpurun_out/pmc_f32_write.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_b16_fetch -o run -- python3 $B16 > gpurun_out/pmc_b16_fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_b16_write -o run -- python3 $B16 > gpurun_out/pmc_b16_write.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/pmc_f32_fetch gpurun_out/pmc_f32_write gpurun_out/round2_conv_traffic.json > gpurun_out/pmc_f32_summary.txt || exit 1
python3 tools/pmc_traffic.py gpurun_out/pmc_b16_fetch gpurun_out/pmc_b16_write gpurun_out/round2_bf16_conv_traffic.json > gpurun_out/pmc_b16_summary.txt || exit 1
for DT in bf16 fp32; do
  SH="--dtype $DT --trunks bathy --shape 128,128,3,1,1,32 --reps 3 --only fwd --fused"
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_${DT}_sq1 -o run -- python3 tools/conv_bench.py $SH > gpurun_out/pmc_${DT}_sq1.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_${DT}_sq2 -o run -- python3 tools/conv_bench.py $SH > gpurun_out/pmc_${DT}_sq2.log 2>&1 || exit 1
done
cat gpurun_out/pmc_f32_summary.txt gpurun_out/pmc_b16_summary.txt
echo done
