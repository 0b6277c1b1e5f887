# session 4: fused batch fit (k_fit_sup_fu) parity + A/B against k_fit_sup + k_fit_update
set -o pipefail
mkdir -p gpurun_out/s4
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_queue.py -k "fit_superposition or configs2 or bench_headline or queue or optimize" -x -v --timeout 300 --timeout-method thread > gpurun_out/s4/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s4/pytest.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for r in 1 2; do
  for f in fu plain; do
    timeout -k 10 300 env MDG_FITSUP=$f python bench.py --no-configs --no-cpu-baseline --verify 1 > gpurun_out/s4/q_${f}_$r.json 2> gpurun_out/s4/q_${f}_$r.err || exit $?
    python -c "
import json;d=json.loads(open('gpurun_out/s4/q_${f}_$r.json').read().strip().splitlines()[-1]);r=d['roofline']
print('$f r$r', round(d['value']), d['verified']['verified'], r['kernel'], round(r['avg_launch_ms'],3), round(r['in_queue']['avg_launch_ms'],3), {k: round(v*1e3,2) for k,v in d['stages_ms_per_spectrum'].items()})"
  done
done
bash tools/ab_libs.sh "gp4 gp8" > gpurun_out/s4/ab.log 2>&1; cat gpurun_out/s4/ab.log
