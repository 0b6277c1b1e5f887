set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 900 python bench.py > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
grep '^{' gpurun_out/bench_full.log > gpurun_out/bench_full.json
python - <<'P'
import json
d=json.load(open('gpurun_out/bench_full.json'))
print('value',d['value'],'lat',d['latency_ms'],'inflight',d['latency_in_stream_ms'],'cpu',d['cpu_baseline']['value'],d['cpu_baseline']['cores'], d['speedup_vs_cpu'])
for k,v in d.get('configs',{}).items(): print(k, v['value'], v.get('speedup_vs_cpu'), (v.get('roofline') or {}).get('kernel'), (v.get('roofline') or {}).get('frac'))
P
