#!/bin/bash
# configs[4] inside bench.py: alone, and with the other configs (bench.py measures it
# first since round 2; before, after configs[0] and [2], its sets took 5.5 ms, not 3.9)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c4o
for c in "4 --steps 24" "0,2,3,4 --steps 24"; do
  tag=$(echo $c | tr ' ,' '__')
  timeout -k 10 300 python bench.py --no-cpu-baseline --configs $c > gpurun_out/c4o/$tag.json 2>/dev/null || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/c4o/$tag.json').read().strip().splitlines()[-1])
print('configs $c:', {k: round(v['value']) for k, v in d['configs'].items()}, 'headline', round(d['value']))"
done
