# session 3: default bench (all configs, both configs[4] environments), lanes test
set -o pipefail
mkdir -p gpurun_out/s3
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "lanes or python_api" -x -v --timeout 120 --timeout-method thread > gpurun_out/s3/pytest.log 2>&1; echo "pytest rc=$?"
timeout -k 10 600 python bench.py > gpurun_out/s3/bench.json 2> gpurun_out/s3/bench.err; echo "bench rc=$?"
python - <<'P'
import json
d=json.loads(open('gpurun_out/s3/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['verified']['verified'], d['batch_latency_ms'])
for k,v in d.get('configs',{}).items(): print(k, v.get('value'), v.get('lanes'), v.get('hw_queues'), v.get('speedup_vs_cpu'), v.get('same_result_as_cpu'))
print(d['cpu_baseline']['value'], d.get('speedup_vs_cpu'))
P
