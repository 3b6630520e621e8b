#!/bin/bash
# round-5 GPU call 10: SQ counters of conv_expand16 vs conv_pipe16 on the f16 inference chunk's
# layer-2 / layer-3 conv3 shapes (two --pmc passes each, conv_bench --shape)
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c10; mkdir -p $O
P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
P2="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
for shape in 128,512,1,1,0,32 256,1024,1,1,0,16; do
  for mode in 0 1; do
    for pass in 1 2; do
      if [ $pass = 1 ]; then C=$P1; else C=$P2; fi
      d=$O/s${shape//,/_}_m${mode}_p$pass
      timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $d -o run -- python3 tools/conv_bench.py --shape $shape --only fwd --fused --dtype f16 --G 20 --B 256 --reps 2 --trunks bathy --expand16 $mode > $d.log 2>&1 || { echo "fail $d"; exit 1; }
    done
  done
done
python3 tools/sq_shapes.py $O/sq.json \
  exp128=$O/s128_512_1_1_0_32_m1_p1,$O/s128_512_1_1_0_32_m1_p2 pipe128=$O/s128_512_1_1_0_32_m0_p1,$O/s128_512_1_1_0_32_m0_p2 \
  exp256=$O/s256_1024_1_1_0_16_m1_p1,$O/s256_1024_1_1_0_16_m1_p2 pipe256=$O/s256_1024_1_1_0_16_m0_p1,$O/s256_1024_1_1_0_16_m0_p2
echo done
