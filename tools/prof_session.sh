#!/bin/bash
# rocprofv3 kernel-trace/stats of bench.py (one config per call); outputs under gpurun_out/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_$tag" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "gpurun_out/prof_$tag.log" 2>&1
rc=$?
echo "prof $tag rc=$rc"
tail -3 "gpurun_out/prof_$tag.log"
exit $rc
