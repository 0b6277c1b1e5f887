#!/bin/bash
# Fit choice by batch size: parity of the fit kernels, default choice per B, full bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s10
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_queue.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s10/tests.log 2>&1 || { tail -30 gpurun_out/s10/tests.log; exit 1; }
tail -2 gpurun_out/s10/tests.log
for B in 1 2 4 8 16 24 32; do
  out=gpurun_out/s10/b$B.json
  timeout -k 10 120 python bench.py --mode stream --batch $B --streams 1 --steps 4 --warmup 1 --no-configs --no-cpu-baseline > $out 2> ${out%.json}.err || { echo "B=$B rc=$?"; exit 1; }
  python -c "
import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); st=d['stages_ms_per_spectrum']
print('B=$B fit us/spectrum', round(1e3*st.get('fit_superposition',0)+1e3*st.get('fit_update',0),2), 'latency ms', round(d['latency_ms'],3), 'spectra/s', round(d['value']))"
done
timeout -k 10 600 python bench.py > gpurun_out/s10/bench.json 2> gpurun_out/s10/bench.err || exit 1
tail -c 3000 gpurun_out/s10/bench.json
