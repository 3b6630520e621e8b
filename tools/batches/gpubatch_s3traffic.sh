# per-shape HBM traffic of both conv families at the bench shapes (G=5, B=64, lazy BN on load)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for dt in fp32 bf16; do
  C="tools/conv_bench.py --dtype $dt --fused --mark --reps 2 --top 5"
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/s3t_${dt}_f -o run -- python3 $C > gpurun_out/s3t_${dt}_f.log 2>&1 || { tail -5 gpurun_out/s3t_${dt}_f.log; exit 1; }
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/s3t_${dt}_w -o run -- python3 $C > gpurun_out/s3t_${dt}_w.log 2>&1 || { tail -5 gpurun_out/s3t_${dt}_w.log; exit 1; }
  python3 tools/shape_traffic.py gpurun_out/s3t_${dt}_f.log gpurun_out/s3t_${dt}_f gpurun_out/s3t_${dt}_w gpurun_out/s3t_${dt}.json > gpurun_out/s3t_${dt}.txt || exit 1
  rm -rf gpurun_out/s3t_${dt}_f gpurun_out/s3t_${dt}_w
done
cat gpurun_out/s3t_fp32.txt gpurun_out/s3t_bf16.txt
