# round 2g: the bench's configs[4] per-GPU slices (S=128/512, B=32) and num_mc=12 leg, then the
# full default bench line that carries them
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --no-roofline --no-bf16 --no-infer > gpurun_out/g_sweep.log 2>&1 || { tail -20 gpurun_out/g_sweep.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/g_sweep.log').read().strip().splitlines()[-1]);print(d['value'], json.dumps(d['train_sweep']))"
timeout -k 10 600 python -u bench.py > gpurun_out/round2g_bench.log 2>&1 || { tail -20 gpurun_out/round2g_bench.log; exit 1; }
tail -1 gpurun_out/round2g_bench.log > gpurun_out/round2g_bench.json
python3 -c "import json;d=json.load(open('gpurun_out/round2g_bench.json'));print(d['value'], d['bf16_train']['value'], d['inference']['value'], json.dumps(d['train_sweep']))"
timeout -k 10 300 python -u tools/infer_chunk.py 50 100 50 100 > gpurun_out/g_chunk.log 2>&1 || { tail -20 gpurun_out/g_chunk.log; exit 1; }
cat gpurun_out/g_chunk.log | grep chunk
