# session 7: default bench (driver form) + force-dist world 1 (gather to rank 0 over RCCL)
set -o pipefail
mkdir -p gpurun_out/s7
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s7/driver_form.json 2> gpurun_out/s7/driver_form.err; echo "bench rc=$?"
python - <<'P'
import json
d=json.loads(open('gpurun_out/s7/driver_form.json').read().strip().splitlines()[-1])
r=d['roofline']
print(d['value'], d['verified']['verified'], d['batch_latency_ms'], r['kernel'], r['frac'], r.get('issue_roofline',{}).get('frac'), r.get('issue_pmc'), d['roofline_pipeline']['frac'])
for k,v in d.get('configs',{}).items(): print(k, v.get('value'), v.get('speedup_vs_cpu'))
print('cpu', d['cpu_baseline']['value'], d.get('speedup_vs_cpu'))
P
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --force-dist --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/s7/forcedist.json 2> gpurun_out/s7/forcedist.err; echo "forcedist rc=$?"
python -c "
import json;d=json.loads(open('gpurun_out/s7/forcedist.json').read().strip().splitlines()[-1])
print(d['value'], d['verified']['verified'], d['rccl_gather_ms']); print(json.dumps(d.get('configs_dist'))[:1500])"
