# acc-start centring with the centre loaded ahead of the tiles + deferred pending-BN staging:
# the 16-bit tests, then kernel statistics and wall clock against the previous library (abtmp/)
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
O=gpurun_out/r6
timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 300 --timeout-method thread -m gpu \
  tests/test_centre16_gpu.py tests/test_fold_gpu.py tests/test_big16_gpu.py tests/test_expand16_gpu.py \
  tests/test_haloc16_gpu.py tests/test_halo16_gpu.py tests/test_kernels16_gpu.py \
  > $O/r6k_tests.log 2>&1; r=$?; tail -2 $O/r6k_tests.log; [ $r -eq 0 ] || { grep -E "FAILED|Error" $O/r6k_tests.log | head -20; exit 1; }
C="--steps 1 --warmup 0 --no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer-sweep --no-bf16 --no-infer-fp32"
MAUV_LIB=$PWD/abtmp/libmauv_head.so MAUV_CENTRE_Y=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hd0 -o run -- python3 bench.py $C > $O/hd0.log 2>&1 || exit 1
MAUV_CENTRE_Y=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/nw0 -o run -- python3 bench.py $C > $O/nw0.log 2>&1 || exit 1
MAUV_CENTRE_Y=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/nw1 -o run -- python3 bench.py $C > $O/nw1.log 2>&1 || exit 1
python3 tools/kstat_diff.py $O/hd0 $O/nw0 20 > $O/r6k_kdiff_head0_new0.txt
python3 tools/kstat_diff.py $O/nw0 $O/nw1 20 > $O/r6k_kdiff_new0_new1.txt
python3 tools/kstat_diff.py $O/hd0 $O/nw1 20 > $O/r6k_kdiff_head0_new1.txt
head -12 $O/r6k_kdiff_*.txt
for arm in "head 0" "new 0" "new 1" "head 0" "new 1"; do
  set -- $arm
  L=""; [ $1 = head ] && L=$PWD/abtmp/libmauv_head.so
  if [ -n "$L" ]; then export MAUV_LIB=$L; else unset MAUV_LIB; fi
  MAUV_CENTRE_Y=$2 timeout -k 10 300 python -u tools/fold_ab.py --flag CENTRE_Y --only $2 --rounds 2 > $O/r6k_wall_$1_$2.txt 2>&1 || exit 1
  echo "$1 centre=$2: $(grep best $O/r6k_wall_$1_$2.txt)"
done
