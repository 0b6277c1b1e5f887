#!/bin/bash
# Marginal cost of each stage in the headline stream mode (16 contexts): the bench's
# value with the stage skipped or shortened (MDG_DIAG_SKIP makes results wrong, so
# the bench's status check is the only check left; diagnostics only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python bench.py --no-configs --no-cpu-baseline --no-profile --steps 480"
one() {  # one <name> <env...> -- <extra bench args>
  local name=$1; shift
  local envs=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
  [ "$1" = "--" ] && shift
  env "${envs[@]}" timeout -k 10 120 $B "$@" > "gpurun_out/decomp_$name.json" 2> "gpurun_out/decomp_$name.err"
  local rc=$?
  echo "$name rc=$rc $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value'],1), round(d['latency_ms'],3))" "gpurun_out/decomp_$name.json" 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
}
for v in "$@"; do
  case "$v" in
    base) one base -- ;;
    nosmooth) one nosmooth MDG_DIAG_SKIP=smooth -- ;;
    nomse) one nomse MDG_DIAG_SKIP=mse -- ;;
    fit1) one fit1 -- --fit-iterations 1 ;;
    noexcl) one noexcl MDG_CHAIN_EXCL=0 -- ;;
    b2) one b2 -- --batch 2 --streams 16 --steps 240 ;;
    b4) one b4 -- --batch 4 --streams 16 --steps 120 ;;
    b16) one b16 -- --batch 16 --streams 16 --steps 32 ;;
    pad5) one pad5 MDG_DIAG_PAD=5 -- ;;
    pad10) one pad10 MDG_DIAG_PAD=10 -- ;;
    pad10s) one pad10s MDG_DIAG_PAD=10 MDG_DIAG_PAD_SMALL=1 -- ;;
    pad10w*) one "$v" MDG_DIAG_PAD=10 MDG_DIAG_PAD_WGS="${v#pad10w}" -- ;;
    nograph) one nograph MDG_GRAPHS=0 -- ;;
    kdev) one kdev HIP_FORCE_DEV_KERNARG=1 -- ;;
    kdev0) one kdev0 HIP_FORCE_DEV_KERNARG=0 -- ;;
    kdevg) one kdevg HIP_FORCE_DEV_KERNARG=1 MDG_GRAPHS=1 -- ;;
    nograph16) one nograph16 MDG_GRAPHS=0 -- --streams 16 ;;
    nograph24) one nograph24 MDG_GRAPHS=0 -- --streams 24 ;;
    fit_*) one "$v" MDG_FITSUP="${v#fit_}" -- ;;
    s[0-9]*) one "$v" -- --streams "${v#s}" ;;
    dup_*) one "$v" MDG_DIAG_DUP="${v#dup_}" -- ;;
    noexcl_dup_smooth) one "$v" MDG_CHAIN_EXCL=0 MDG_DIAG_DUP=smooth -- ;;
    *) echo "unknown $v" ;;
  esac
done
