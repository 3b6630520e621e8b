#!/bin/bash
# round-5 GPU call 13: the block-output fold per shape at the f16 inference chunk (G = 20, B = 256)
# against the unfused pair, and SQ counters of the fold on a layer-1 and a layer-2 shape
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c13; mkdir -p $O
timeout -k 10 300 python -u tools/fold_bench.py --dtype f16 --G 20 --B 256 > $O/fold_bench.log 2>&1 || { echo "bench failed"; exit 1; }
P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
P2="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
for shape in 256,64,64 512,128,32 1024,256,16; do
  for pass in 1 2; do
    if [ $pass = 1 ]; then C=$P1; else C=$P2; fi
    d=$O/s${shape//,/_}_p$pass
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $d -o run -- python3 tools/fold_bench.py --shape $shape --only-fold --dtype f16 --G 20 --B 256 --reps 2 > $d.log 2>&1 || { echo "fail $d"; exit 1; }
  done
done
python3 tools/sq_shapes.py $O/sq.json l1=$O/s256_64_64_p1,$O/s256_64_64_p2 l2=$O/s512_128_32_p1,$O/s512_128_32_p2 l3=$O/s1024_256_16_p1,$O/s1024_256_16_p2
echo done
