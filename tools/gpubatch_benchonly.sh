set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/bo_bench.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/bo_bench.log').read().strip().splitlines()[-1]);print(d['value'], d['inference']['value'], d['bf16_train']['value'], d['fp32_exact_mfma']['value'], d['roofline']['frac'])"
echo done
