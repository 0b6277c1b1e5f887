#!/bin/bash
# A/B comparisons and sweeps of bench.py configurations in one GPU session: one
# bench run per configuration and round (rounds alternate the configurations), one
# summary line each: spectra/s, verification, latency, the fit kernel alone and in
# the queue, per-stage us per spectrum.
#
# Usage (GPU box): [ROUNDS=2] [BENCH="--steps 6"] bash tools/ab.sh <tag> "<name> [ENV=VAL ...] [bench flags]" ...
#   ENV=VAL entries set the environment (MDG_FITSUP=tw7, MDG_TW_G=98, MDG_MSE_NPT=1,
#   MDGPU_LIB=build/libmdgpu_x.so MDGPU_ALLOW_STALE=1 for another build of the engine,
#   GPU_MAX_HW_QUEUES=32 ...); everything else goes to bench.py, e.g.
#     "b4_tw7 MDG_FITSUP=tw7 --mode stream --batch 4 --streams 1 --steps 4 --warmup 1"
#     "q192 --max-batch 192 --lanes 2"
#     "c4_l8 MDGPU_LANES=8 --c4-only"
# Every run gets --no-configs --no-cpu-baseline. Results: gpurun_out/ab_<tag>/, summary
# in gpurun_out/ab_<tag>/summary.txt. Stops at the first run that fails.
# (Replaces the round-2/3 one-off wrappers: sweep.sh, ab_lib.sh, ab_libs.sh,
# fit_by_batch*.sh, c4_lanes.sh and the gpu_s*.sh sessions.)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
dir=gpurun_out/ab_$tag
mkdir -p "$dir"
cfgs=("$@")
for r in $(seq 1 "${ROUNDS:-1}"); do
  for cfg in "${cfgs[@]}"; do
    set -- $cfg
    name=$1; shift
    envs=(); flags=()
    for a in "$@"; do
      case "$a" in --*) flags+=("$a") ;; *=*) envs+=("$a") ;; *) flags+=("$a") ;; esac
    done
    out=$dir/${name}_r$r.json
    timeout -k 10 "${AB_TIMEOUT:-300}" env "${envs[@]}" python bench.py --no-configs --no-cpu-baseline \
        $BENCH "${flags[@]}" > "$out" 2> "${out%.json}.err"
    rc=$?
    python - "$out" "$name r$r" "$rc" >> "$dir/summary.txt" <<'P'
import json, sys
path, name, rc = sys.argv[1:]
try:
    d = json.loads(open(path).read().strip().splitlines()[-1])
except Exception as e:
    print(f"{name}: rc={rc} ({e})", flush=True)
    sys.exit()
r = d.get("roofline") or {}
st = d.get("stages_ms_per_spectrum", {})
fit = 1e3 * (st.get("fit_superposition", 0) + st.get("fit_update", 0))
parts = [f"{name}: {d['value']:.0f} spectra/s"]
if isinstance(d.get("verified"), dict):
    parts.append(f"verified {d['verified'].get('verified')}")
if d.get("latency_ms") is not None:
    parts.append(f"latency {d['latency_ms']:.3f} ms")
if r.get("avg_launch_ms") is not None:
    q = (r.get("in_queue") or {}).get("avg_launch_ms")
    parts.append(f"{r.get('kernel')} {r['avg_launch_ms']:.3f} ms" + (f" (in queue {q:.3f})" if q else ""))
if st:
    parts.append(f"fit {fit:.1f} us/spectrum; " + ", ".join(f"{k} {v * 1e3:.2f}" for k, v in st.items()))
print(", ".join(parts), flush=True)
P
    tail -1 "$dir/summary.txt"
    if [ $rc -ne 0 ]; then echo "stop ($name rc=$rc)"; exit $rc; fi
  done
done
