set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --configs 4 --no-cpu-baseline --steps 60 > gpurun_out/bench_c4.log 2>&1 || { tail -20 gpurun_out/bench_c4.log; exit 1; }
python - <<'P'
import json
d=json.loads([l for l in open('gpurun_out/bench_c4.log') if l.startswith('{')][0])
print('value',d['value'])
for k,v in d.get('configs',{}).items(): print(k, v['value'], v['ms_per_step'], (v.get('roofline') or {}).get('kernel'))
P
