# configs[4] (16 blood spectra, Python surface, host buffers) by lane count and
# hardware queues: bench.py --c4-only under each environment
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c4
for q in 4 32; do
  for l in 1 2 3 4 8 16; do
    [ $l -ge $q ] && continue
    timeout -k 10 200 env GPU_MAX_HW_QUEUES=$q MDGPU_LANES=$l python bench.py --c4-only > gpurun_out/c4/q${q}_l$l.json 2> gpurun_out/c4/q${q}_l$l.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/c4/q${q}_l$l.json').read().strip().splitlines()[-1]); print('queues $q lanes', d['lanes'], round(d['value']), 'spectra/s', round(d['ms_per_step'],2), 'ms/set')"
  done
done
