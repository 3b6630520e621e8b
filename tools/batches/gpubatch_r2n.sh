set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_host.py > gpurun_out/r2n_h.log 2>&1 || { tail -20 gpurun_out/r2n_h.log; exit 1; }
cat gpurun_out/r2n_h.log
