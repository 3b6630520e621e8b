# round 3: per-shape tables of every conv pass on the current library — training slices (G=5,
# B=64, lazy BN on load as in the step) for bf16 and fp32, and an f16 inference chunk (G=10,
# B=256, forwards)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/conv_bench.py --dtype bf16 --fused --top 600 > gpurun_out/r3sh_bf16.txt 2>&1 || { tail -5 gpurun_out/r3sh_bf16.txt; exit 1; }
tail -4 gpurun_out/r3sh_bf16.txt
timeout -k 10 300 python -u tools/conv_bench.py --dtype fp32 --fused --top 600 > gpurun_out/r3sh_fp32.txt 2>&1 || { tail -5 gpurun_out/r3sh_fp32.txt; exit 1; }
tail -4 gpurun_out/r3sh_fp32.txt
timeout -k 10 300 python -u tools/conv_bench.py --dtype f16 --fused --G 10 --B 256 --only fwd --top 600 > gpurun_out/r3sh_f16inf.txt 2>&1 || { tail -5 gpurun_out/r3sh_f16inf.txt; exit 1; }
tail -2 gpurun_out/r3sh_f16inf.txt
echo done
