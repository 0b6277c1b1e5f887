set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "concurrent_contexts" --timeout 240 --timeout-method thread > gpurun_out/pytest_cc.log 2>&1 || { tail -30 gpurun_out/pytest_cc.log; exit 1; }
tail -2 gpurun_out/pytest_cc.log
timeout -k 10 600 python bench.py --configs 4 --no-cpu-baseline --steps 60 > gpurun_out/bench_c4.log 2>&1 || { tail -20 gpurun_out/bench_c4.log; exit 1; }
python -c "import json;d=json.loads([l for l in open('gpurun_out/bench_c4.log') if l.startswith('{')][0]);v=d['configs']['configs[4]'];print(v['value'], v['roofline']['kernel'], v['roofline']['frac'], v['roofline']['avg_launch_ms'])"
