set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/pt_all.log 2>&1 || { tail -30 gpurun_out/pt_all.log; exit 1; }
tail -2 gpurun_out/pt_all.log
for io in copy direct copy direct; do
  F=""; [ $io = copy ] && F="--copy-io"
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-configs --no-profile --steps 400 $F > gpurun_out/io.log 2>&1 || exit $?
  python -c "import json;d=json.loads([l for l in open('gpurun_out/io.log') if l.startswith('{')][0]);print('$io', round(d['value']), round(d['latency_ms'],3), round(d['host_submit_ms_per_step'],4))"
done
