#!/bin/bash
# round-5 GPU call 17: SQ counters of conv_haloc16 (mode 1: 32 x 64 wave tiles, mode 2: 64 x 64)
# against the implicit GEMM (mode 0) on the f16 layer-2 / layer-3 conv2 shapes
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c17; mkdir -p $O
P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
P2="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
for shape in 128,128,3,1,1,32 256,256,3,1,1,16; do
  for mode in 0 1 2; do
    for pass in 1 2; do
      if [ $pass = 1 ]; then C=$P1; else C=$P2; fi
      d=$O/s${shape//,/_}_m${mode}_p$pass
      timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $d -o run -- python3 tools/conv_bench.py --shape $shape --only fwd --fused --dtype f16 --G 5 --B 256 --reps 2 --trunks bathy --haloc16 $mode > $d.log 2>&1 || { echo "fail $d"; exit 1; }
    done
  done
done
A=""
for shape in 128_128_3_1_1_32 256_256_3_1_1_16; do for mode in 0 1 2; do A="$A c${shape%%_*}m$mode=$O/s${shape}_m${mode}_p1,$O/s${shape}_m${mode}_p2"; done; done
python3 tools/sq_shapes.py $O/sq.json $A
echo done
