set -o pipefail
mkdir -p gpurun_out/cd2 gpurun_out/sim3
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all3.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_all3.log
[ $rc -eq 0 ] || exit $rc
for n in 2048 131072; do timeout -k 5 60 tools/ubench/chain_diag 1 3 0 $n > gpurun_out/cd2/n$n.txt 2>&1 || exit 3; done
timeout -k 10 120 python -u tools/c0_breakdown.py --sim 300 > gpurun_out/sim3/breakdown.txt 2>&1 || exit 3
timeout -k 10 120 python -u tools/c0_breakdown.py 100 > gpurun_out/sim3/breakdown_blood.txt 2>&1 || exit 3
for b in 1 16; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sim3/bt$b -o run -- python3 tools/blood_trace.py --sim $b > gpurun_out/sim3/bt$b.log 2>&1 || exit 3
  python tools/blood_trace.py --summary $(find gpurun_out/sim3/bt$b -name run_kernel_trace.csv | head -1) > gpurun_out/sim3/bt$b.txt
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sim3/blood$b -o run -- python3 tools/blood_trace.py $b > gpurun_out/sim3/blood$b.log 2>&1 || exit 3
  python tools/blood_trace.py --summary $(find gpurun_out/sim3/blood$b -name run_kernel_trace.csv | head -1) > gpurun_out/sim3/blood$b.txt
done
