# A/B: eight-wave 32x64 wave tiles (default) vs four-wave 64x64 wave tiles, one or two accumulators
set -o pipefail
mkdir -p gpurun_out
run() { timeout -k 10 200 python -u tools/conv_bench.py --dtype fp32 --top 3 --trunks bathy > gpurun_out/w4_$1.log 2>&1 || exit 1; echo "$1 $(grep 'TOTAL all' gpurun_out/w4_$1.log)"; }
run default
MAUV_SPLIT_W8=0 MAUV_F32_MATH=split1 run w4_one
MAUV_SPLIT_W8=0 run w4_two
MAUV_SPLIT_W8=1 run w8_128only
echo done
