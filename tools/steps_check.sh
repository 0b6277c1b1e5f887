set -o pipefail
mkdir -p gpurun_out/steps
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-configs --no-cpu-baseline > gpurun_out/steps/driver_r$r.json 2> gpurun_out/steps/driver_r$r.err || exit $?
  timeout -k 10 300 python bench.py --no-configs --no-cpu-baseline > gpurun_out/steps/default_r$r.json 2> gpurun_out/steps/default_r$r.err || exit $?
  timeout -k 10 300 python bench.py --no-configs --no-cpu-baseline --steps 1 --warmup 5 > gpurun_out/steps/oneround_r$r.json 2> gpurun_out/steps/oneround_r$r.err || exit $?
done
for f in gpurun_out/steps/*.json; do python -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), d['steps'], round(d['ms_per_step'],3), d['config']['spectra_per_gpu_per_step'])"; done
