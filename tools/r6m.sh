# deferred pending-BN staging in the split-fp32 kernel: fp32 kernel tests, then per-kernel time
# and wall clock of the fp32 / bf16 training steps against the previous library (abtmp/)
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
O=gpurun_out/r6
timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 300 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_f32_math_gpu.py tests/test_bwd_fusion_gpu.py tests/test_fold_gpu.py \
  > $O/r6m_tests.log 2>&1; r=$?; tail -2 $O/r6m_tests.log; [ $r -eq 0 ] || { grep -E "FAILED|Error" $O/r6m_tests.log | head -20; exit 1; }
C="--steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer"
HL=$PWD/abtmp/libmauv_head.so
MAUV_TRUNK_STREAMS=0 MAUV_LIB=$HL MAUV_CENTRE_Y=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t32h -o run -- python3 bench.py $C --no-bf16 > $O/t32h.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t32n -o run -- python3 bench.py $C --no-bf16 > $O/t32n.log 2>&1 || exit 1
python3 tools/steady_stats.py $O/t32h $O/r6m_fp32_steady_head.csv && python3 tools/steady_stats.py $O/t32n $O/r6m_fp32_steady_new.csv || exit 1
python3 tools/kstat_diff.py $O/t32h $O/t32n 20 > $O/r6m_kdiff_fp32_head_new.txt; head -14 $O/r6m_kdiff_fp32_head_new.txt
for arm in "head 0 fp32" "new 1 fp32" "head 0 fp32" "new 1 fp32" "head 0 bf16" "new 1 bf16" "head 0 bf16" "new 1 bf16"; do
  set -- $arm
  if [ $1 = head ]; then export MAUV_LIB=$HL; else unset MAUV_LIB; fi
  MAUV_CENTRE_Y=$2 timeout -k 10 300 python -u tools/fold_ab.py --train --dtype $3 --flag CENTRE_Y --only $2 --rounds 2 --steps 8 > $O/r6m_wall.txt 2>&1 || exit 1
  echo "$1 centre=$2 $3: $(grep best $O/r6m_wall.txt)"
done
