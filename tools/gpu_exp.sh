#!/bin/bash
# E-step / step-tail experiments: GPU parity tests, bench, kernel stats
mkdir -p gpurun_out; : > gpurun_out/status.log
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/status.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
step pytest_gpu 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread
step bench_grid 240 python bench.py --steps 10 --warmup 5 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof; mkdir -p gpurun_out/prof
step prof_stats 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/stats -o stats --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-hbm-copy
