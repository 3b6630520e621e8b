mkdir -p gpurun_out/r6
export TMPDIR=/tmp
O=gpurun_out/r6
for c in 1 0; do
timeout -k 10 300 python -u tools/pred_bisect.py --seeds 8 --no-fit --S-opt 64 --S-son 64 --B 8 --N 4 --centre $c > $O/pred_sweep_randinit_c$c.log 2>&1; r=$?; grep -E "variance|over" $O/pred_sweep_randinit_c$c.log | tail -9; [ $r -eq 0 ] || exit 1
done
