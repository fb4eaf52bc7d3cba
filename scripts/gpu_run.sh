#!/bin/bash
# Runs a sequence of GPU steps on the gpurun box; stops at the first fault/timeout
# (exit codes 124/134/137/139 or signals), continues past ordinary test failures.
# usage: scripts/gpu_run.sh "<name>:<timeout>:<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; tmo="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (timeout ${tmo}s): $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  case $rc in
    0|1|2) ;;
    *) echo "stopping after fault/timeout in $name"; exit $rc ;;
  esac
done
