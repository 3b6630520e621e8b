# per-shape conv timings with algorithmic bytes and the per-launch roofline (max of MFMA and
# HBM time): f16 forwards at an inference-like chunk (G=10 MC groups of B=256), bf16 and fp32
# training passes at the bench's G=5, B=64 (lazy BN on load, statistics epilogue)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/conv_bench.py --dtype f16 --G 10 --B 256 --only fwd --fused --top 40 > gpurun_out/s3_shapes_f16.txt 2>&1 || { tail -20 gpurun_out/s3_shapes_f16.txt; exit 1; }
timeout -k 10 240 python -u tools/conv_bench.py --dtype bf16 --fused --top 60 > gpurun_out/s3_shapes_bf16.txt 2>&1 || { tail -20 gpurun_out/s3_shapes_bf16.txt; exit 1; }
timeout -k 10 300 python -u tools/conv_bench.py --dtype fp32 --fused --top 60 > gpurun_out/s3_shapes_f32.txt 2>&1 || { tail -20 gpurun_out/s3_shapes_f32.txt; exit 1; }
tail -4 gpurun_out/s3_shapes_f16.txt gpurun_out/s3_shapes_bf16.txt gpurun_out/s3_shapes_f32.txt
