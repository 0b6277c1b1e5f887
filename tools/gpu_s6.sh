# session 6: work-queue fit (k_fit_sup_dyn) parity + A/B against k_fit_sup
set -o pipefail
mkdir -p gpurun_out/s6
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "fit_superposition" -x -v --timeout 200 --timeout-method thread > gpurun_out/s6/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/s6/pytest.log | tail -2
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 env MDG_FITSUP=dyn python -u -m pytest tests/test_gpu_configs.py -k configs2 -x -v --timeout 250 --timeout-method thread > gpurun_out/s6/pytest_c2.log 2>&1; rc=$?; echo "configs2 dyn rc=$rc"; tail -1 gpurun_out/s6/pytest_c2.log
[ $rc -ne 0 ] && exit $rc
run() {  # tag env...
  local tag=$1; shift
  timeout -k 10 300 env "$@" python bench.py --max-batch 256 --lanes 2 --steps 6 --no-configs --no-cpu-baseline --verify 1 > gpurun_out/s6/q_$tag.json 2> gpurun_out/s6/q_$tag.err || exit $?
  python -c "
import json;d=json.loads(open('gpurun_out/s6/q_$tag.json').read().strip().splitlines()[-1]);r=d['roofline']
print('$tag', round(d['value']), d['verified']['verified'], r['kernel'], round(r['avg_launch_ms'],3), round(r['in_queue']['avg_launch_ms'],3), round(r['issue_roofline']['frac'],3), {k: round(v*1e3,2) for k,v in d['stages_ms_per_spectrum'].items()})"
}
for r in 1 2; do
  run plain_$r MDG_FITSUP=plain
  run dyn_$r MDG_FITSUP=dyn
  run dyn_w5_$r MDG_FITSUP=dyn MDG_DYN_WPC=5
  run dyn_p8_$r MDG_FITSUP=dyn MDG_DYN_PIECES=8
done
