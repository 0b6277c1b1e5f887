#!/bin/bash
# rocprofv3 runs of bench.py (headline only); outputs under gpurun_out/prof_<tag>*/
#   trace <tag> [bench args]          kernel trace + stats
#   pmc <tag> <COUNTER> [bench args]  one PMC counter pass (never with sys/runtime traces)
#   calib <COUNTER>                   the FETCH/WRITE width calibration (tools/ubench/fetch_calib)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
mode=$1; tag=$2; shift 2
if [ "$mode" = trace ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_$tag" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-configs "$@" > "gpurun_out/prof_$tag.log" 2>&1
elif [ "$mode" = calib ]; then
  timeout -s KILL 120 rocprofv3 --pmc "$tag" --output-format csv -d "$ROOT/gpurun_out/prof_calib_$tag" -o run -- "$ROOT/tools/ubench/fetch_calib" > "gpurun_out/prof_calib_$tag.log" 2>&1
else
  ctr=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$ctr" --output-format csv -d "$ROOT/gpurun_out/prof_${tag}_$ctr" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-configs --no-profile "$@" > "gpurun_out/prof_${tag}_$ctr.log" 2>&1
fi
rc=$?
echo "prof $mode $tag rc=$rc"
tail -2 gpurun_out/prof_*"$tag"*.log
exit $rc
