# Fit kernel by batch size (stream mode, one context, batches back to back): the
# fit stage per spectrum alone and the batch latency, for each MDG_FITSUP choice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fitb
for B in 4 8 12 16 24 32 48 64; do
  for f in dpp plain tf tw7; do
    out=gpurun_out/fitb/b${B}_$f.json
    timeout -k 10 120 env MDG_FITSUP=$f python bench.py --mode stream --batch $B --streams 1 --steps 4 --warmup 1 --no-configs --no-cpu-baseline > $out 2> ${out%.json}.err || { echo "B=$B $f rc=$?"; continue; }
    python -c "
import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); st=d['stages_ms_per_spectrum']
print('B=$B $f', 'fit us/spectrum', round(1e3*st.get('fit_superposition',0)+1e3*st.get('fit_update',0),2), 'latency ms', round(d['latency_ms'],3), 'spectra/s', round(d['value']))"
  done
done
