set -o pipefail
mkdir -p gpurun_out
for E in 1 0; do for S in 8 16 24; do
  MDG_CHAIN_EXCL=$E timeout -k 10 300 python bench.py --streams $S --steps 480 --no-cpu-baseline --no-configs --no-profile > gpurun_out/ex_$E.log 2>&1 || exit $?
  python -c "import json;d=json.loads([l for l in open('gpurun_out/ex_$E.log') if l.startswith('{')][0]);print('excl $E S $S', round(d['value']), round(d['latency_ms'],3))"
done; done
