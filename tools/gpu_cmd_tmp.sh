set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for F in tf tw7; do
  MDG_FITSUP=$F timeout -k 10 600 python bench.py --configs 4 --no-cpu-baseline --steps 60 > gpurun_out/c4.log 2>&1 || exit $?
  python -c "import json;d=json.loads([l for l in open('gpurun_out/c4.log') if l.startswith('{')][0]);v=d['configs']['configs[4]'];print('$F', round(v['value']), round(v['ms_per_step'],3))"
done; done
