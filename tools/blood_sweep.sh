#!/bin/bash
# Fit-kernel sweep on blood batches (GPU box): for each B and each MDG_FITSUP value,
# one rocprofv3 kernel trace of tools/blood_trace.py B; prints the fit kernel's mean
# launch time. Usage: bash tools/blood_sweep.sh "<B ...>" "<kernel ...>" [ENV=VAL ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/bs
Bs=$1; Ks=$2; shift 2
for b in $Bs; do for k in $Ks; do
  d=gpurun_out/bs/${k}_$b
  env "$@" MDG_FITSUP=$k timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- \
      python3 tools/blood_trace.py $b > $d.log 2>&1 || exit 1
  echo "B=$b $k: $(python3 tools/blood_trace.py --brief $(find $d -name '*kernel_trace.csv' | head -1) | grep -o 'fit_sup[^(]*' | head -3 | tr '\n' ' ')"
done; done | tee -a gpurun_out/bs/summary.txt
