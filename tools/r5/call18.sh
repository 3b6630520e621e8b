#!/bin/bash
# round-5 GPU call 18: conv_haloc16 with per-thread offsets fixed over the chunks (scalar
# chunk / tap offsets): tests, per-shape A/B of the unroll / wave-tile variants (experimental
# modes 1-4), SQ counters of the default form on the layer-3 shape
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c18; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 300 --timeout-method thread tests/test_haloc16_gpu.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; [ $r -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/haloc_ab.py --dtype bf16 > $O/ab_bf16.log 2>&1; r=$?; echo "ab bf16 rc=$r"; [ $r -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/haloc_ab.py --dtype f16 --B 256 > $O/ab_f16.log 2>&1; r=$?; echo "ab f16 rc=$r"; [ $r -eq 0 ] || exit 1
P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
P2="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
A=""
for mode in 1 3; do
  for pass in 1 2; do
    if [ $pass = 1 ]; then C=$P1; else C=$P2; fi
    d=$O/s256_m${mode}_p$pass
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $d -o run -- python3 tools/conv_bench.py --shape 256,256,3,1,1,16 --only fwd --fused --dtype f16 --G 5 --B 256 --reps 2 --trunks bathy --haloc16 $mode > $d.log 2>&1 || { echo "fail $d"; exit 1; }
  done
  A="$A c256m$mode=$O/s256_m${mode}_p1,$O/s256_m${mode}_p2"
done
python3 tools/sq_shapes.py $O/sq.json $A
echo done
