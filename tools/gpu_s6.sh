# session 6: work-queue fit (k_fit_sup_dyn) parity + A/B
set -o pipefail
mkdir -p gpurun_out/s6
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "fit_superposition" -x -v --timeout 200 --timeout-method thread > gpurun_out/s6/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "dyn|passed|failed" gpurun_out/s6/pytest.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 env MDG_FITSUP=dyn python -u -m pytest tests/test_gpu_configs.py -k configs2 -x -v --timeout 250 --timeout-method thread > gpurun_out/s6/pytest_c2.log 2>&1; rc=$?; echo "configs2 dyn rc=$rc"; tail -3 gpurun_out/s6/pytest_c2.log
for r in 1 2; do
  for f in plain dyn; do
    timeout -k 10 300 env MDG_FITSUP=$f python bench.py --max-batch 256 --lanes 2 --steps 6 --no-configs --no-cpu-baseline --verify 1 > gpurun_out/s6/q_${f}_$r.json 2> gpurun_out/s6/q_${f}_$r.err || exit $?
    python -c "
import json;d=json.loads(open('gpurun_out/s6/q_${f}_$r.json').read().strip().splitlines()[-1]);r=d['roofline']
print('$f r$r', round(d['value']), d['verified']['verified'], r['kernel'], round(r['avg_launch_ms'],3), round(r['in_queue']['avg_launch_ms'],3), round(r['issue_roofline']['frac'],3), {k: round(v*1e3,2) for k,v in d['stages_ms_per_spectrum'].items()})"
  done
done
