# session 8: queue tests (flush deadline), the round's profile set, configs[4] lanes sweep
set -o pipefail
mkdir -p gpurun_out/s8
timeout -k 10 600 python -u -m pytest tests/test_gpu_queue.py -x -v --timeout 300 --timeout-method thread > gpurun_out/s8/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/s8/pytest.log | tail -2
[ $rc -ne 0 ] && exit $rc
bash tools/prof_all.sh > gpurun_out/prof_all.log 2>&1; rc=$?; grep "rc=" gpurun_out/prof_all.log; [ $rc -ne 0 ] && exit $rc
bash tools/c4_lanes.sh
