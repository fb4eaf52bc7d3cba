#!/bin/bash
# PMC passes over one command (each pass its own rocprofv3 run; counters only
# with --kernel-trace, never with runtime/sys traces).
# usage: [PASSES="fetch write"] scripts/pmc.sh <outname> <script.py | executable> [args...]
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/$1"; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  echo "=== pmc pass $name: $*"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d "$out/$name" -o "$name" --output-format csv \
    -- "${CMD[@]}" > "$out/$name.log" 2>&1
  local rc=$?
  echo "=== pass $name rc=$rc"
  return $rc
}
ARGS=("$@")
# a .py script runs under python3; anything else is an executable in the repo
if [[ "${ARGS[0]}" == *.py ]]; then CMD=(python3 "$root/${ARGS[0]}" "${ARGS[@]:1}")
else CMD=("$root/${ARGS[0]}" "${ARGS[@]:1}"); fi
PASSES="${PASSES:-sq lds tcc fetch write ta}"
rc=0
for p in $PASSES; do
  case $p in
    sq) pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES ;;
    lds) pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM ;;
    tcc) pass tcc TCC_HIT_sum TCC_MISS_sum ;;
    fetch) pass fetch FETCH_SIZE ;;
    write) pass write WRITE_SIZE ;;
    ta) pass ta TA_TA_BUSY_sum TA_BUSY_avr ;;
  esac
  rc=$?
  # stop at the first failing pass (a fault or timeout must end the GPU work)
  [ $rc -ne 0 ] && exit $rc
done
exit 0
