set -o pipefail
mkdir -p gpurun_out/s2
timeout -k 10 600 python -u -m pytest tests/test_gpu_ignore_regions.py tests/test_gpu_queue.py -x -v --timeout 300 --timeout-method thread > gpurun_out/s2/pytest.log 2>&1; echo "pytest rc=$?"
for cfg in "128 2" "128 3" "256 2" "96 3" "64 4" "192 2"; do
  set -- $cfg
  timeout -k 10 240 python bench.py --max-batch $1 --lanes $2 --steps 8 --warmup 2 --no-configs --no-cpu-baseline --verify 1 > gpurun_out/s2/q_$1_$2.json 2> gpurun_out/s2/q_$1_$2.err
  rc=$?; echo "q $1 x $2 rc=$rc"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  python -c "import json;d=json.loads(open('gpurun_out/s2/q_$1_$2.json').read().strip().splitlines()[-1]);print(d['value'], d['batch_latency_ms'], d['verified']['verified'], d['roofline']['issue_roofline']['frac'] if d['roofline'] else None, d['roofline_pipeline']['frac'])"
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --force-dist --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/s2/forcedist.json 2> gpurun_out/s2/forcedist.err; echo "forcedist rc=$?"
tail -c 3000 gpurun_out/s2/forcedist.json
