# library A/B against abtmp/libmauv_head.so (the previous commit's build): tests, bitwise equality,
# per-kernel time and wall clock of the training steps
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
O=gpurun_out/r6
HL=$PWD/abtmp/libmauv_head.so
timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 300 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_kernels16_gpu.py tests/test_bwd_fusion_gpu.py tests/test_fold_gpu.py \
  > $O/r6n_tests.log 2>&1; r=$?; tail -2 $O/r6n_tests.log; [ $r -eq 0 ] || { grep -E "FAILED|Error" $O/r6n_tests.log | head -20; exit 1; }
for d in bf16 fp32; do
  MAUV_LIB=$HL timeout -k 10 300 python -u tools/lib_bitcmp.py save /tmp/bc_head_$d.pt $d || exit 1
  timeout -k 10 300 python -u tools/lib_bitcmp.py save /tmp/bc_new_$d.pt $d || exit 1
  python tools/lib_bitcmp.py cmp /tmp/bc_head_$d.pt /tmp/bc_new_$d.pt | tee -a $O/r6n_bitcmp.txt
done
C="--steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer"
MAUV_TRUNK_STREAMS=0 MAUV_LIB=$HL timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b16h -o run -- python3 bench.py $C --dtype bf16 --no-bf16 > $O/b16h.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b16n -o run -- python3 bench.py $C --dtype bf16 --no-bf16 > $O/b16n.log 2>&1 || exit 1
python3 tools/steady_stats.py $O/b16h $O/r6n_bf16_steady_head.csv && python3 tools/steady_stats.py $O/b16n $O/r6n_bf16_steady_new.csv || exit 1
python3 tools/kstat_diff.py $O/b16h $O/b16n 16 > $O/r6n_kdiff_bf16_head_new.txt; head -14 $O/r6n_kdiff_bf16_head_new.txt
for arm in "head bf16" "new bf16" "head bf16" "new bf16" "head fp32" "new fp32" "head fp32" "new fp32"; do
  set -- $arm
  if [ $1 = head ]; then export MAUV_LIB=$HL; else unset MAUV_LIB; fi
  timeout -k 10 300 python -u tools/fold_ab.py --train --dtype $2 --flag CENTRE_Y --only 1 --rounds 2 --steps 8 > $O/r6n_wall.txt 2>&1 || exit 1
  echo "$1 $2: $(grep best $O/r6n_wall.txt)" | tee -a $O/r6n_wall_all.txt
done
