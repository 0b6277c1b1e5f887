set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for S in 3 4; do
  timeout -k 10 300 python bench.py --streams $S --steps 60 --no-cpu-baseline --no-configs > gpurun_out/streams_$S.log 2>&1 || exit $?
  python -c "import json;d=json.loads([l for l in open('gpurun_out/streams_$S.log') if l.startswith('{')][0]);print($S, d['value'], d['latency_ms'])"
done
timeout -k 10 900 python bench.py --steps 60 > gpurun_out/bench_full.log 2>&1 || exit $?
python - <<'P'
import json
d=json.loads([l for l in open('gpurun_out/bench_full.log') if l.startswith('{')][0])
print('value',d['value'],'lat',d['latency_ms'],'cpu',d['cpu_baseline']['value'],d['cpu_baseline']['cores'])
for k,v in d.get('configs',{}).items(): print(k, v['value'], v.get('speedup_vs_cpu'), (v.get('roofline') or {}).get('kernel'))
print(d['cpu_baselines'])
P
