#!/bin/bash
# GPU session driver: each GPU step under its own time limit; stop at the first
# crash/timeout (exit >= 124 or signal), continue after plain test failures.
mkdir -p gpurun_out
step() {
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "stopping after $name (rc=$rc)"; exit $rc
  fi
  return 0
}
