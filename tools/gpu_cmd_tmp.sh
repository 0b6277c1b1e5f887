set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/mfma_experiment.py 256 > gpurun_out/mfma_experiment.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/mfma_experiment.log | tail -5
exit $rc
