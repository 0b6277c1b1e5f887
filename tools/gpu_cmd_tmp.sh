set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 600 --timeout-method thread --durations=5 > gpurun_out/pytest_configs.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_configs.log
exit $rc
