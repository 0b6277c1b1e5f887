#!/bin/bash
# One GPU session: smoke, GPU tests, benches. Stops at the first GPU fault/abort/timeout
# (exit codes other than 0/1); a plain test failure (1) does not stop the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log" | tee -a gpurun_out/session.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)" | tee -a gpurun_out/session.log; exit $rc; fi
  return 0
}
for step in "$@"; do
  case "$step" in
    smoke) run smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    tests_all) run pytest_gpu 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    bench) run bench1 600 python bench.py ;;
    driver) run driver_form 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    forcedist) run forcedist 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --force-dist --steps 4 --warmup 1 --no-cpu-baseline ;;
    stream) run stream18 300 python bench.py --mode stream --no-configs --no-cpu-baseline ;;
    bench64) run bench64 600 python bench.py --mode stream --batch 64 --streams 1 --steps 5 --warmup 1 --no-cpu-baseline ;;
    bench256) run bench256 600 python bench.py --mode stream --batch 256 --streams 1 --steps 3 --warmup 1 --no-cpu-baseline ;;
    *) echo "unknown step $step" ;;
  esac
done
