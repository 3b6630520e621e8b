# 16-bit epilogue: the previous dx of an accumulating data gradient prefetched (addend slot);
# against the previous commit's library (abtmp/libmauv_head.so)
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
O=gpurun_out/r6
HL=$PWD/abtmp/libmauv_head.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_kernels16_gpu.py tests/test_haloc16_gpu.py tests/test_halo16_gpu.py tests/test_model16_gpu.py > $O/r6x_tests.log 2>&1; r=$?; tail -1 $O/r6x_tests.log; [ $r -eq 0 ] || { grep -E "FAILED|Error" $O/r6x_tests.log | head -20; exit 1; }
MAUV_LIB=$HL timeout -k 10 300 python -u tools/lib_bitcmp.py save /tmp/bc_head_bf16.pt bf16 || exit 1
timeout -k 10 300 python -u tools/lib_bitcmp.py save /tmp/bc_new_bf16.pt bf16 || exit 1
python tools/lib_bitcmp.py cmp /tmp/bc_head_bf16.pt /tmp/bc_new_bf16.pt
C="--steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer --no-bf16 --dtype bf16"
MAUV_TRUNK_STREAMS=0 MAUV_LIB=$HL timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/x16h -o run -- python3 bench.py $C > $O/x16h.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/x16n -o run -- python3 bench.py $C > $O/x16n.log 2>&1 || exit 1
python3 tools/kstat_diff.py $O/x16h $O/x16n 8
for arm in head new head new; do
  if [ $arm = head ]; then export MAUV_LIB=$HL; else unset MAUV_LIB; fi
  timeout -k 10 300 python -u tools/fold_ab.py --train --dtype bf16 --flag CENTRE_Y --only 1 --rounds 2 --steps 6 > $O/r6x_wall.txt 2>&1 || exit 1
  echo "$arm bf16: $(grep best $O/r6x_wall.txt)"
done
