#!/bin/bash
# GPU parity suite + smoke (+ optional extra steps given as arguments, each "NAME SECONDS CMD...").
# Every step has its own time limit; the first failing step ends the script (no GPU work after a
# fault, abort or timeout).  Logs: gpurun_out/<name>.log, summary: gpurun_out/status.log.
mkdir -p gpurun_out; : > gpurun_out/status.log
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/status.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step pytest_gpu ${PYTEST_SECS:-900} python -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
# one optional extra step: NAME SECONDS CMD...
if [ $# -ge 3 ]; then step "$@"; fi
