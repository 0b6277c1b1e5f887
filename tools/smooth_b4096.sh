#!/bin/bash
# smoother kernels on the configs[3] batch (4096 x 65536): stage time per step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for k in "$@"; do
  MDG_SMOOTH=$k timeout -k 10 200 python bench.py --no-configs --no-cpu-baseline --batch 4096 --n 65536 --peaks 1024 --hw-scale 2 --cap 2048 --streams 1 --steps 1 --warmup 1 > gpurun_out/sm4096_$k.json 2> gpurun_out/sm4096_$k.err || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); st=d['stages_ms_per_spectrum']; print(sys.argv[2], round(d['value'],1), 'smooth_ms_per_step', round(st['smooth']*4096,3))" gpurun_out/sm4096_$k.json $k
done
