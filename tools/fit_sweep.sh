#!/bin/bash
# Fit-superposition kernel sweep: bench stage times per kernel choice and batch size.
# usage (GPU box): bash tools/fit_sweep.sh "dpp tf plain" "1 2 8 16"
out=gpurun_out/fit_sweep.txt; : > $out
for b in $2; do for k in $1; do
  MDG_FITSUP=$k timeout -k 10 120 python bench.py --batch $b --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/fs.json 2>/dev/null || exit 1
  python - "$k" "$b" >> $out <<'PY'
import json,sys
d=json.loads(open('gpurun_out/fs.json').read().strip().splitlines()[-1])
st=d['stages_ms_per_step']
print(sys.argv[1], 'B=',sys.argv[2], 'spectra/s=%.1f'%d['value'], 'fit_sup_ms=%.4f'%st['fit_superposition'], 'mse_ms=%.4f'%st['mse_superposition'])
PY
  tail -1 $out
done; done
