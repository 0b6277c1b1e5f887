set -o pipefail
# smoother parity on the variant build first, then the A/B
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "smooth" > gpurun_out/pytest_scb.log 2>&1 || { tail -20 gpurun_out/pytest_scb.log; exit 1; }
tail -1 gpurun_out/pytest_scb.log
bash tools/ab_lib.sh
