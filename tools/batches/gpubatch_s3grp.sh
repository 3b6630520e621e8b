# weight-gradient block order: the G groups of one pixel slice adjacent (MAUV_XCD_GRID=2: the
# stems' shared im2col rows read into one L2 once) vs slices of one group adjacent (1)
set -o pipefail
mkdir -p gpurun_out
B="--no-cpu-baseline --exact-steps 0 --no-roofline --no-infer"
for v in 1 2 1 2; do
  MAUV_XCD_GRID=$v timeout -k 10 300 python -u bench.py $B > gpurun_out/s3g_tr.log 2>&1 || { tail -5 gpurun_out/s3g_tr.log; exit 1; }
  echo "grid=$v train"; tail -1 gpurun_out/s3g_tr.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['bf16_train']['value'])"
done
for v in 1 2; do
  MAUV_XCD_GRID=$v MAUV_TRUNK_STREAMS=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --exact-steps 0 --no-infer --steps 2 --warmup 1 > gpurun_out/s3g_rf.log 2>&1 || { tail -5 gpurun_out/s3g_rf.log; exit 1; }
  echo "grid=$v serial conv ms/step"; tail -1 gpurun_out/s3g_rf.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['conv_ms_per_step'], d['bf16_train']['roofline']['conv_ms_per_step'])"
done
