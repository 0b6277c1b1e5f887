set -o pipefail
mkdir -p gpurun_out
for S in 2 3 4 6; do
  timeout -k 10 300 python bench.py --streams $S --steps 80 --no-cpu-baseline --no-configs > gpurun_out/streams_$S.log 2>&1 || exit $?
  python -c "import json;d=json.loads([l for l in open('gpurun_out/streams_$S.log') if l.startswith('{')][0]);print($S, d['value'], d['latency_ms'])"
done
for S in 3 4; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --streams $S --steps 80 --no-cpu-baseline --no-configs > gpurun_out/streams_q8_$S.log 2>&1 || exit $?
  python -c "import json;d=json.loads([l for l in open('gpurun_out/streams_q8_$S.log') if l.startswith('{')][0]);print('q8', $S, d['value'], d['latency_ms'])"
done
