#!/bin/bash
# Round measurement: GPU tests, smoke, the default bench line (with cpu_baseline), then profiles.
# PROF_PASSES selects the rocprofv3 passes of tools/gpu_prof.sh (default: all).
mkdir -p gpurun_out; : > gpurun_out/status.log
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/status.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step pytest_gpu 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py
step prof 1000 bash tools/gpu_prof.sh
