set -o pipefail
mkdir -p gpurun_out
for ab in 0 1 2 3 4 6; do
  for sh in 128,128,3,1,1,32 256,1024,1,1,0,16 64,64,3,1,1,64; do
    echo "abl $ab shape $sh" >> gpurun_out/abl.log
    MAUV_SPLIT_ABLATE=$ab timeout -k 10 120 python -u tools/conv_bench.py --trunks opt --shape $sh --reps 5 | grep -v ids >> gpurun_out/abl.log 2>&1 || exit 1
  done
done
