# library GEMM vs the 16-bit implicit-GEMM conv on the same M x N x K (tools/gemm_probe.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_probe.py --dtype f16 --G 10 --B 256 > gpurun_out/s3_probe_f16.txt 2>&1 || { tail -20 gpurun_out/s3_probe_f16.txt; exit 1; }
timeout -k 10 300 python -u tools/gemm_probe.py --dtype bf16 --G 5 --B 64 > gpurun_out/s3_probe_bf16.txt 2>&1 || { tail -20 gpurun_out/s3_probe_bf16.txt; exit 1; }
cat gpurun_out/s3_probe_f16.txt gpurun_out/s3_probe_bf16.txt
