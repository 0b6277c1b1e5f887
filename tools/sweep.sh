#!/bin/bash
# Parameterised sweep of the round-2 stream mode (--mode stream): one bench.py run per configuration, one summary line
# each. Replaces the round-2 one-off wrappers (stream_batch_sweep.sh, idle_streams.sh,
# fit_stream_sweep.sh, ...).
#
# Usage (GPU box): bash tools/sweep.sh <tag> "<cfg>" ["<cfg>" ...]
#   cfg = "B S [extra bench.py flags / ENV=VAL ...]"   B spectra per call, S contexts
#   total spectra per run ~ $SPECTRA (default 1536); results gpurun_out/sweep_<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
dir=gpurun_out/sweep_$tag
mkdir -p "$dir"
SPECTRA=${SPECTRA:-1536}
i=0
for cfg in "$@"; do
  set -- $cfg
  B=$1; S=$2; shift 2
  envs=(); flags=()
  for a in "$@"; do
    case "$a" in *=*) [[ "$a" == --* ]] && flags+=("$a") || envs+=("$a") ;; *) flags+=("$a") ;; esac
  done
  K=$(( SPECTRA / (B * S) )); [ $K -lt 2 ] && K=2
  i=$((i + 1))
  out=$dir/$i.json
  echo "== [$i] B=$B S=$S K=$K ${envs[*]} ${flags[*]}" >> "$dir/summary.txt"
  timeout -k 10 240 env "${envs[@]}" python bench.py --mode stream --batch "$B" --streams "$S" --steps "$K" \
      --warmup 2 --no-configs --no-cpu-baseline --no-profile "${flags[@]}" > "$out" 2> "${out%.json}.err"
  rc=$?
  python - "$out" "$B" "$S" "$rc" "${envs[*]} ${flags[*]}" >> "$dir/summary.txt" <<'EOF'
import json, sys
path, B, S, rc, extra = sys.argv[1:]
try:
    d = json.loads(open(path).read().strip().splitlines()[-1])
    print(f"B={B} S={S} {extra}: {d['value']:.0f} spectra/s, {d['ms_per_step']:.3f} ms/step, "
          f"latency {d['latency_ms']:.3f} ms", flush=True)
except Exception as e:
    print(f"B={B} S={S} {extra}: rc={rc} ({e})", flush=True)
EOF
  tail -1 "$dir/summary.txt"
  if [ $rc -ne 0 ]; then echo "stop (rc=$rc)"; exit $rc; fi
done
