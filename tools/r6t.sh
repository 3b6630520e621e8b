# every split-fp32 SEQ (short-K) kernel with register double-buffered stages at the pipelined
# kernel's register budget (abtmp/libmauv_seqD.so) against this library: fp32 step kernel time
# and wall clock, and bitwise equality of one step
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
O=gpurun_out/r6
VD=$PWD/abtmp/libmauv_seqD.so
timeout -k 10 300 python -u tools/lib_bitcmp.py save /tmp/bc_cur_fp32.pt fp32 || exit 1
MAUV_LIB=$VD timeout -k 10 300 python -u tools/lib_bitcmp.py save /tmp/bc_d_fp32.pt fp32 || exit 1
python tools/lib_bitcmp.py cmp /tmp/bc_cur_fp32.pt /tmp/bc_d_fp32.pt
C="--steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-sweep --no-infer --no-bf16"
MAUV_TRUNK_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t32c -o run -- python3 bench.py $C > $O/t32c.log 2>&1 || exit 1
MAUV_TRUNK_STREAMS=0 MAUV_LIB=$VD timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t32d -o run -- python3 bench.py $C > $O/t32d.log 2>&1 || exit 1
python3 tools/kstat_diff.py $O/t32c $O/t32d 8
for arm in cur D cur D; do
  if [ $arm = D ]; then export MAUV_LIB=$VD; else unset MAUV_LIB; fi
  timeout -k 10 300 python -u tools/fold_ab.py --train --dtype fp32 --flag CENTRE_Y --only 1 --rounds 2 --steps 6 > $O/r6t_wall.txt 2>&1 || exit 1
  echo "$arm fp32: $(grep best $O/r6t_wall.txt)"
done
