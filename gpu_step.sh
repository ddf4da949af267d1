#!/bin/bash
# Runs GPU steps in order, each under its own timeout; stops at the first crash/timeout
# (exit codes other than 0 = pass, 1 = pytest test failures).
mkdir -p gpurun_out
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
