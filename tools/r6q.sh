# bn_bwd_partial row batch for 16-bit storage: 4 rows (this library, 136 VGPRs) vs 3 / 2
# (abtmp/libmauv_ru{3,2}.so, 120 / 104 VGPRs): kernel statistics of the serial bf16 step
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
O=gpurun_out/r6
C="--steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer --no-bf16 --dtype bf16"
for v in cur ru6 ru8 cap; do
  if [ $v = cur ]; then unset MAUV_LIB; else export MAUV_LIB=$PWD/abtmp/libmauv_$v.so; fi
  MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/q_$v -o run -- python3 bench.py $C > $O/q_$v.log 2>&1 || exit 1
  echo "$v: $(grep bn_bwd_partial $O/q_$v/run_kernel_stats.csv | cut -d, -f1-6)" | tee -a $O/r6q.txt
done
unset MAUV_LIB
for v in ru6 ru8 cap; do python3 tools/kstat_diff.py $O/q_cur $O/q_$v 4; done
