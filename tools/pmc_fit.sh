#!/bin/bash
# Small-batch fit diagnostics (GPU box): rocprofv3 PMC passes of tools/blood_trace.py B
# (the blood set through one context, B spectra per call), one counter group per run,
# a kernel trace of the same command for the durations, then the stamped
# microbenchmark tools/ubench/fit_diag (built on the CPU with -DMDG_DIAG).
#   bash tools/pmc_fit.sh [B] [fit_diag args ...]
# Outputs under gpurun_out/pmcfit_b<B>/ (PMCFIT_TAG overrides the suffix); summarise
# with tools/pmc_groups.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B=${1:-16}
O=gpurun_out/pmcfit${PMCFIT_TAG:-_b$B}
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1
echo "list rc=$?"
# keep only the counters this box lists (an unknown name would fail the pass)
pick() {
  local out=()
  for c in "$@"; do grep -qw "$c" $O/avail.txt && out+=("$c"); done
  echo "${out[@]}"
}
A=$(pick GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU)
L=$(pick GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA)
M=$(pick SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_IFETCH)
echo "A: $A"; echo "L: $L"; echo "M: $M"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/blood_trace.py $B > $O/trace.log 2>&1 || exit $?
for g in A L M; do
  ctrs=${!g}
  [ -n "$ctrs" ] || continue
  timeout -s KILL 180 rocprofv3 --pmc $ctrs --output-format csv -d $O/pmc_$g -o run -- python3 tools/blood_trace.py $B > $O/pmc_$g.log 2>&1
  rc=$?
  echo "pmc $g rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
shift
if [ $# -gt 0 ] && [ -x tools/ubench/fit_diag ]; then
  timeout -k 10 120 tools/ubench/fit_diag "$@" > $O/fit_diag.log 2>&1
  echo "fit_diag rc=$?"
fi
