set -o pipefail
mkdir -p gpurun_out
for f in 0 1; do
  MAUV_DGRAD_BN_EPILOGUE=$f timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-infer --no-bf16 --exact-steps 0 --steps 5 --warmup 1 > gpurun_out/fl_$f.log 2>&1 || exit 1
done
echo done
