set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_g48.log 2>&1 || { tail -20 gpurun_out/pytest_g48.log; exit 1; }
tail -1 gpurun_out/pytest_g48.log
bash tools/ab_lib.sh
