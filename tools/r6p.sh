# fp32 BN backward row batch sizes: this library (partial 4 rows, apply 2) against a build with
# 2 / 1 rows for fp32 storage (abtmp/libmauv_varB.so): kernel statistics and wall clock
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
O=gpurun_out/r6
VB=$PWD/abtmp/libmauv_varB.so
C="--steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer --no-bf16"
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/f32a -o run -- python3 bench.py $C > $O/f32a.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 MAUV_LIB=$VB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/f32b -o run -- python3 bench.py $C > $O/f32b.log 2>&1 || exit 1
python3 tools/kstat_diff.py $O/f32a $O/f32b 8 > $O/r6p_kdiff_f32.txt; cat $O/r6p_kdiff_f32.txt
for arm in "cur" "varB" "cur" "varB"; do
  if [ $arm = varB ]; then export MAUV_LIB=$VB; else unset MAUV_LIB; fi
  timeout -k 10 300 python -u tools/fold_ab.py --train --dtype fp32 --flag CENTRE_Y --only 1 --rounds 2 --steps 6 > $O/r6p_wall.txt 2>&1 || exit 1
  echo "$arm fp32: $(grep best $O/r6p_wall.txt)" | tee -a $O/r6p_wall_all.txt
done
