# session 9: MSE recurrence + 512-point tiles: parity, then A/B in the queue
set -o pipefail
mkdir -p gpurun_out/s9
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "mse or golden or configs2 or lanes or chunked" -x -v --timeout 300 --timeout-method thread > gpurun_out/s9/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/s9/pytest.log | tail -2
[ $rc -ne 0 ] && exit $rc
run() {  # tag env...
  local tag=$1; shift
  timeout -k 10 300 env "$@" python bench.py --steps 6 --no-configs --no-cpu-baseline --verify 1 > gpurun_out/s9/q_$tag.json 2> gpurun_out/s9/q_$tag.err || exit $?
  python -c "
import json;d=json.loads(open('gpurun_out/s9/q_$tag.json').read().strip().splitlines()[-1]);r=d['roofline']
print('$tag', round(d['value']), d['verified']['verified'], {k: round(v*1e3,2) for k,v in d['stages_ms_per_spectrum'].items()})"
}
for r in 1 2; do
  run npt1_$r MDG_MSE_NPT=1
  run npt2_$r MDG_MSE_NPT=2
done
