# session 5: queue shape sweep (value, fit alone / in queue) + fit group-size variants
set -o pipefail
mkdir -p gpurun_out/s5
for cfg in "192 2" "256 2" "384 2" "256 1" "128 2" "192 2" "256 2"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --max-batch $1 --lanes $2 --steps 6 --no-configs --no-cpu-baseline --verify 1 > gpurun_out/s5/q_$1_$2.json 2> gpurun_out/s5/q_$1_$2.err || exit $?
  python -c "
import json;d=json.loads(open('gpurun_out/s5/q_$1_$2.json').read().strip().splitlines()[-1]);r=d['roofline']
print('$1x$2', round(d['value']), d['verified']['verified'], round(r['avg_launch_ms'],3), round(r['in_queue']['avg_launch_ms'],3), round(r['issue_roofline']['frac'],3), {k: round(v*1e3,2) for k,v in d['stages_ms_per_spectrum'].items()})"
done
bash tools/ab_libs.sh "gp4 gp8" > gpurun_out/s5/ab.log 2>&1; cat gpurun_out/s5/ab.log
