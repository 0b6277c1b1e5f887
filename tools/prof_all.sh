#!/bin/bash
# Full profile set for one round (GPU box): kernel traces + stats and the two PMC
# passes (FETCH_SIZE, WRITE_SIZE; one counter per run) of
#   q256         the headline: queue mode, 256-spectrum batches on 2 lanes
#   b256         configs[2]: one 256-spectrum batch per step (stream mode, 1 context)
#   b4096_n65536 configs[3] on one GPU
# then tools/pmc_summary.py / tools/trace_summary.py turn them into profiles/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
S=tools/prof_session.sh
bash $S trace q256 --steps 6 --warmup 2 --verify 0
bash $S pmc q256 FETCH_SIZE --steps 2 --warmup 1 --verify 0
bash $S pmc q256 WRITE_SIZE --steps 2 --warmup 1 --verify 0
bash $S trace b256 --mode stream --batch 256 --streams 1 --steps 2 --warmup 1
bash $S pmc b256 FETCH_SIZE --mode stream --batch 256 --streams 1 --steps 1 --warmup 1
bash $S pmc b256 WRITE_SIZE --mode stream --batch 256 --streams 1 --steps 1 --warmup 1
bash $S trace b4096_n65536 --mode stream --batch 4096 --streams 1 --steps 1 --warmup 1 --n 65536 --peaks 1024 --hw-scale 2 --cap 2048
