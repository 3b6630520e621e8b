set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_g9.py > gpurun_out/r2n_c.log 2>&1 || { tail -20 gpurun_out/r2n_c.log; exit 1; }
MAUV_STEM_GEMM=0 timeout -k 10 300 python -u tools/diag_g9.py > gpurun_out/r2n_d.log 2>&1 || { tail -20 gpurun_out/r2n_d.log; exit 1; }
head -4 gpurun_out/r2n_c.log; tail -7 gpurun_out/r2n_c.log; head -4 gpurun_out/r2n_d.log
