#!/bin/bash
# E-step / step-tail experiments: GPU parity tests, bench, stamps
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
STC_LIB=spark-text-clustering_amd/stc/libstc_stamp.so step stamp_grid 240 python tools/stamp_estep.py
