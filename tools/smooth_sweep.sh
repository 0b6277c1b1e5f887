#!/bin/bash
# smoother kernels by batch size: smooth stage ms per step (131072-point spectra)
#   bash tools/smooth_sweep.sh "B1 B2 ..." "kernel1 kernel2 ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in $1; do
  for k in $2; do
    MDG_SMOOTH=$k timeout -k 10 200 python bench.py --no-configs --no-cpu-baseline --batch $b --streams 1 --steps 1 --warmup 1 > gpurun_out/sw_${b}_$k.json 2> gpurun_out/sw_${b}_$k.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); st=d['stages_ms_per_spectrum']; b=int(sys.argv[3]); print('B', b, sys.argv[2], round(d['value'],1), 'smooth_ms', round(st['smooth']*b,3), d['roofline']['kernel'] if d['roofline']['stage']=='smooth' else '')" gpurun_out/sw_${b}_$k.json $k $b
  done
done
