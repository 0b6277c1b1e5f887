#!/bin/bash
# A/B of engine builds in one session (GPU box): the in-tree library against
# build/libmdgpu_<tag>.so variants (same sources, other -D flags), headline bench
# alternating, two rounds. Usage: bash tools/ab_libs.sh "<tags>" [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
tags=$1; shift
mkdir -p gpurun_out/ab
for r in 1 2; do
  for t in tree $tags; do
    if [ $t = tree ]; then lib=(env); else lib=(env MDGPU_LIB=$ROOT/build/libmdgpu_$t.so); fi
    out=gpurun_out/ab/${t}_r$r.json
    timeout -k 10 300 "${lib[@]}" python bench.py --no-configs --no-cpu-baseline --verify 1 "$@" > $out 2> ${out%.json}.err || exit $?
    python - "$out" "$t r$r" <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
st = d.get("stages_ms_per_spectrum", {})
print(f"{sys.argv[2]}: {d['value']:.0f} spectra/s verified {d['verified']['verified']} fit alone "
      f"{r.get('avg_launch_ms', 0):.3f} ms, in queue {r.get('in_queue', {}).get('avg_launch_ms', 0):.3f} ms; "
      + ", ".join(f"{k} {v * 1e3:.2f}us" for k, v in st.items()), flush=True)
P
  done
done
