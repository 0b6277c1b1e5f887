set -o pipefail
mkdir -p gpurun_out
for F in 10 5 1; do
  timeout -k 10 300 python bench.py --fit-iterations $F --steps 480 --no-cpu-baseline --no-configs --no-profile > gpurun_out/fi.log 2>&1 || exit $?
  python -c "import json;d=json.loads([l for l in open('gpurun_out/fi.log') if l.startswith('{')][0]);print('fit iters $F', round(d['value']), round(d['latency_ms'],3))"
done
