#!/bin/bash
# Round-end bench evidence: the driver's command line, then the default run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/driver_form.json 2> gpurun_out/final/driver_form.err || exit $?
timeout -k 10 600 python bench.py > gpurun_out/final/default.json 2> gpurun_out/final/default.err || exit $?
for f in gpurun_out/final/*.json; do python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', round(d['value']), 'x cpu', round(d['speedup_vs_cpu'],1), {k: round(v['value']) for k, v in d['configs'].items()})"; done
