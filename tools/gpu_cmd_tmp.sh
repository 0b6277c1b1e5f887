set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "fit_superposition_kernels or golden_case" --timeout 300 --timeout-method thread > gpurun_out/pytest_fit.log 2>&1 || { tail -30 gpurun_out/pytest_fit.log; exit 1; }
tail -2 gpurun_out/pytest_fit.log
timeout -k 10 300 python tools/mse_error.py > gpurun_out/mse_error.log 2>&1 || { tail -20 gpurun_out/mse_error.log; exit 1; }
grep MDG_MSE gpurun_out/mse_error.log
for O in 0 1; do
MDG_MSE_OCT=$O timeout -k 10 300 python bench.py --batch 256 --streams 1 --steps 3 --warmup 1 --no-cpu-baseline --no-configs > gpurun_out/b256_oct$O.log 2>&1 || exit $?
python -c "import json;d=json.loads([l for l in open('gpurun_out/b256_oct$O.log') if l.startswith('{')][0]);print('oct $O b256', round(d['value']), {k:round(v*256,3) for k,v in d['stages_ms_per_spectrum'].items() if v*256>0.5})"
done
for F in tf tq tq11 tq15; do
  MDG_FITSUP=$F GPU_MAX_HW_QUEUES=32 timeout -k 10 120 python tools/stream_diag.py 1 80 > gpurun_out/fit_$F.log 2>&1 || exit $?
  grep -E "S=|fit_sup|mse_sup" gpurun_out/fit_$F.log | tr '\n' ' '; echo " $F"
  MDG_FITSUP=$F timeout -k 10 300 python bench.py --steps 480 --no-cpu-baseline --no-configs --no-profile > gpurun_out/fitb_$F.log 2>&1 || exit $?
  python -c "import json;d=json.loads([l for l in open('gpurun_out/fitb_$F.log') if l.startswith('{')][0]);print('$F', round(d['value']), round(d['latency_ms'],3))"
done
