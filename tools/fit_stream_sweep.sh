#!/bin/bash
# B=1 fit kernel choice under the headline stream: bench.py (20 contexts by default)
# per MDG_FITSUP value, two rounds, plus the fit stage time of one context alone.
# Usage (GPU box): bash tools/fit_stream_sweep.sh "tw7 tw3 tw9 tf" [extra bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fit_stream
kinds=$1; shift
for r in 1 2; do for k in $kinds; do
  out=gpurun_out/fit_stream/${k}_r$r.json
  MDG_FITSUP=$k timeout -k 10 180 python bench.py --no-configs --no-cpu-baseline "$@" > $out 2> ${out%.json}.err || exit $?
  python - "$out" "$k r$r" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = d["stages_ms_per_spectrum"]
print(f"{sys.argv[2]}: {d['value']:.0f} spectra/s, latency {d['latency_ms']:.3f} ms, "
      f"fit {st['fit_superposition'] * 1e3:.1f} us/spectrum alone ({d['roofline']['kernel']})",
      flush=True)
EOF
done; done
