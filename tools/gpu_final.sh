# Round-end evidence (GPU box): the full -m gpu suite, then the driver's bench line.
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/final/pytest_gpu.log | tail -8
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/driver_form.json 2> gpurun_out/final/driver_form.err; rc=$?
echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
python - <<'P'
import json
d = json.loads(open("gpurun_out/final/driver_form.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(round(d["value"]), d["verified"]["verified"], r["kernel"], round(r["frac"], 4), r["traffic"],
      round(r["issue_roofline"]["frac"], 3), round(d["roofline_pipeline"]["frac"], 3),
      round(d["cpu_baseline"]["value"], 1), round(d["speedup_vs_cpu"], 1))
for k, v in d.get("configs", {}).items():
    print(k, v.get("value"), v.get("lanes"), v.get("speedup_vs_cpu"))
P
