# A/B: BN-backward partial sums from the dgrad epilogue (fp32)
set -o pipefail
mkdir -p gpurun_out
for E in 0 1 0 1; do
MAUV_DGRAD_BN_EPILOGUE=$E timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-steps 0 --no-roofline --no-infer --no-bf16 > gpurun_out/dg_$E.log 2>&1 || exit 1
echo "E=$E $(tail -n 1 gpurun_out/dg_$E.log | cut -c90-160)"
done
echo done
