#!/bin/bash
# full profile set for one round: traces and PMC passes at B=1 and B=256
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
bash tools/prof_session.sh trace b1 --steps 10
bash tools/prof_session.sh trace b256 --batch 256 --steps 2 --warmup 1
bash tools/prof_session.sh pmc b1 FETCH_SIZE --steps 5
bash tools/prof_session.sh pmc b1 WRITE_SIZE --steps 5
bash tools/prof_session.sh pmc b256 FETCH_SIZE --batch 256 --steps 1 --warmup 1
bash tools/prof_session.sh pmc b256 WRITE_SIZE --batch 256 --steps 1 --warmup 1
