#!/bin/bash
# MSE stage time at B=1 (single context) and B=256, plus the 20-context stream
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python bench.py --no-configs --no-cpu-baseline --streams 1 --steps 40 > gpurun_out/q_b1.json &&
timeout -k 10 120 python bench.py --no-configs --no-cpu-baseline --streams 1 --batch 256 --steps 2 --warmup 1 > gpurun_out/q_b256.json &&
timeout -k 10 120 python bench.py --no-configs --no-cpu-baseline --no-profile --steps 24 > gpurun_out/q_s20.json &&
python - <<'PY'
import json
for t in ("b1", "b256", "s20"):
    d = json.load(open(f"gpurun_out/q_{t}.json"))
    st = d.get("stages_ms_per_spectrum", {})
    print(t, round(d["value"], 1), "mse_ms", st.get("mse_superposition"), "select_ms", st.get("select"), "lat", round(d["latency_ms"], 3))
PY
