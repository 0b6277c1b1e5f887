#!/bin/bash
# Headline stream with the multi-rank machinery live (RCCL process group at world
# size 1, warm-up and timed gathers) against the plain run: what RCCL's own streams
# cost the contexts' hardware queues.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rccl
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do for s in ${RCCL_STREAMS:-18 20}; do
  out=gpurun_out/rccl/plain_s${s}_r$r.json
  timeout -k 10 200 python bench.py --no-configs --no-cpu-baseline --no-profile --streams $s > $out 2>/dev/null || exit $?
  python -c "import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); print('plain streams $s r$r:', round(d['value']))"
  out=gpurun_out/rccl/dist_s${s}_r$r.json
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=$((29600 + r * 10 + s)) \
      bench.py --force-dist --no-configs --no-cpu-baseline --no-profile --streams $s > $out 2> ${out%.json}.err || exit $?
  python -c "import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); print('rccl  streams $s r$r:', round(d['value']))"
done; done
