#!/bin/bash
# Stream throughput with B spectra per context call (configs[1] spectra), against the
# B=1 headline: does batching inside each stream beat the hardware-queue limit?
# Usage (GPU box): bash tools/stream_batch_sweep.sh  -> gpurun_out/sweep_batch/*.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep_batch
for cfg in "1 20" "2 10" "2 16" "2 20" "4 8" "4 12" "4 16" "8 8"; do
  set -- $cfg
  B=$1; S=$2; K=$(( 480 / (B * S) ))  # rounds of S calls
  out=gpurun_out/sweep_batch/b${B}_s${S}.json
  timeout -k 10 180 python bench.py --batch "$B" --streams "$S" --steps "$K" --warmup 3 \
      --no-configs --no-cpu-baseline --no-profile > "$out" 2> "${out%.json}.err"
  rc=$?
  python - "$out" "$B" "$S" "$rc" <<'EOF'
import json, sys
path, B, S, rc = sys.argv[1:]
try:
    d = json.loads(open(path).read().strip().splitlines()[-1])
    print(f"B={B} streams={S}: {d['value']:.0f} spectra/s, {d['ms_per_step']:.3f} ms/step, "
          f"latency {d['latency_ms']:.3f} ms", flush=True)
except Exception as e:
    print(f"B={B} streams={S}: rc={rc} ({e})", flush=True)
EOF
  if [ $rc -ne 0 ]; then echo "stop (rc=$rc)"; exit $rc; fi
done
