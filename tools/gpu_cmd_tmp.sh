set -o pipefail
mkdir -p gpurun_out
for D in 2 4 8; do
MDG_TWQ_D=$D timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "twq" > gpurun_out/pt_twq.log 2>&1 || { tail -30 gpurun_out/pt_twq.log; exit 1; }
tail -1 gpurun_out/pt_twq.log
MDG_TWQ_D=$D MDG_FITSUP=twq timeout -k 10 300 python bench.py --no-cpu-baseline --no-configs --steps 400 > gpurun_out/twq.log 2>&1 || exit $?
python -c "import json;d=json.loads([l for l in open('gpurun_out/twq.log') if l.startswith('{')][0]);print('D=$D', round(d['value']), round(d['latency_ms'],3), round(d['stages_ms_per_spectrum']['fit_superposition']*1e3,1))"
done
