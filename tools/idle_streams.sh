#!/bin/bash
# Headline stream with K extra idle HIP streams alive (RCCL's streams in a multi-rank
# run are such streams): does the hardware-queue edge move?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/idle
for r in 1 2; do for k in 0 1 2 3 4; do for s in 20 18; do
  out=gpurun_out/idle/k${k}_s${s}_r$r.json
  timeout -k 10 200 python bench.py --no-configs --no-cpu-baseline --no-profile --idle-streams $k --streams $s > $out 2>/dev/null || exit $?
  python -c "
import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); print('idle $k streams $s r$r:', round(d['value']))"
done; done; done
