set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "fit_superposition_kernels" --timeout 120 --timeout-method thread > gpurun_out/pytest_tfq.log 2>&1 || { tail -30 gpurun_out/pytest_tfq.log; exit 1; }
tail -1 gpurun_out/pytest_tfq.log
for F in tf tfq; do
  MDG_FITSUP=$F GPU_MAX_HW_QUEUES=32 timeout -k 10 120 python tools/stream_diag.py 1 80 > gpurun_out/fit_$F.log 2>&1 || exit $?
  grep -E "S=|fit_sup" gpurun_out/fit_$F.log | tr '\n' ' '; echo " $F"
  for S in 1 16 24; do
  MDG_FITSUP=$F timeout -k 10 300 python bench.py --streams $S --steps 480 --no-cpu-baseline --no-configs --no-profile > gpurun_out/fitb_$F.log 2>&1 || exit $?
  python -c "import json;d=json.loads([l for l in open('gpurun_out/fitb_$F.log') if l.startswith('{')][0]);print('$F S $S', round(d['value']), round(d['latency_ms'],3))"
  done
done
