# per-shape conv timings (bench shapes, G=5 B=64): bf16 and fp32, fused as in the model
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/conv_bench.py --dtype bf16 --fused --top 80 > gpurun_out/r2e_bf16.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv_bench.py --dtype fp32 --fused --top 80 > gpurun_out/r2e_fp32.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv_bench.py --dtype f16 --fused --G 20 --B 256 --only fwd --top 60 > gpurun_out/r2e_f16inf.log 2>&1 || exit 1
tail -4 gpurun_out/r2e_bf16.log gpurun_out/r2e_fp32.log gpurun_out/r2e_f16inf.log
