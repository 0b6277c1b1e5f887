# Term-fold fits with one workgroup per tile for every spectrum (MDG_TW_G) against
# the current choice, by batch size (stream mode, one context, back to back).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fitb2
run() {  # B tag env...
  local B=$1 tag=$2; shift 2
  out=gpurun_out/fitb2/b${B}_$tag.json
  timeout -k 10 120 env "$@" python bench.py --mode stream --batch $B --streams 1 --steps 4 --warmup 1 --no-configs --no-cpu-baseline > $out 2> ${out%.json}.err || { echo "B=$B $tag rc=$?"; return; }
  python -c "
import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); st=d['stages_ms_per_spectrum']
print('B=$B $tag', 'fit us/spectrum', round(1e3*st.get('fit_superposition',0)+1e3*st.get('fit_update',0),2), 'latency ms', round(d['latency_ms'],3), 'spectra/s', round(d['value']))"
}
for B in 1 2 4 8 16 32 64 128 256; do
  run $B default
  run $B tw7_g98 MDG_FITSUP=tw7 MDG_TW_G=98
  run $B tf_g256 MDG_FITSUP=tf MDG_TW_G=256
done
