#!/bin/bash
# A/B of two engine builds in one session: build/libmdgpu_base.so (the previous
# sources, MDGPU_ALLOW_STALE) against the in-tree library. Headline stream and the
# one-context stage times, alternating, two rounds.
# Usage (GPU box): [AB_S1_ONLY=1] bash tools/ab_lib.sh [extra bench args]  -> gpurun_out/ab/*.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out/ab
summ() {
  python - "$1" "$2" <<'EOF'
import json, sys
path, tag = sys.argv[1:]
d = json.loads(open(path).read().strip().splitlines()[-1])
st = d.get("stages_ms_per_spectrum", {})
print(f"{tag}: {d['value']:.0f} spectra/s, latency {d['latency_ms']:.3f} ms, "
      + ", ".join(f"{k} {v * 1e3:.1f}us" for k, v in st.items()), flush=True)
EOF
}
for r in 1 2; do
  for which in base new; do
    if [ $which = base ]; then lib=(env MDGPU_LIB=$ROOT/build/libmdgpu_base.so MDGPU_ALLOW_STALE=1); else lib=(env); fi
    out=gpurun_out/ab/${which}_s20_r$r.json
    [ "${AB_S1_ONLY:-0}" = 1 ] || timeout -k 10 180 "${lib[@]}" python bench.py --mode stream --no-configs --no-cpu-baseline "$@" > $out 2> ${out%.json}.err || exit $?
    [ "${AB_S1_ONLY:-0}" = 1 ] || summ $out "$which streams=20 r$r"
    out=gpurun_out/ab/${which}_s1_r$r.json
    timeout -k 10 180 "${lib[@]}" python bench.py --mode stream --no-configs --no-cpu-baseline --streams 1 --steps 40 "$@" > $out 2> ${out%.json}.err || exit $?
    summ $out "$which streams=1 r$r"
  done
done
