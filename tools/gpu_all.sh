#!/bin/bash
# diag + GPU tests + bench (fast path and v1).  A crash/timeout/abort (rc >= 124) ends the script;
# an ordinary failure (e.g. a test assertion, rc 1) is recorded and the next step still runs.
mkdir -p gpurun_out; : > gpurun_out/status.log
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/status.log
  if [ $rc -ge 124 ] || [ $rc -lt 0 ]; then exit $rc; fi
  return 0
}
step diag_wave 240 python tools/diag_wave.py
step pytest_gpu 400 python -m pytest tests -x -q -m gpu
step bench_wave 240 python bench.py --steps 10 --warmup 10 --no-cpu-baseline
STC_DISABLE_WAVE=1 step bench_v1 240 python bench.py --steps 10 --warmup 10 --no-cpu-baseline
STC_WAVE_SHAPE=1 step bench_shape1 240 python bench.py --steps 10 --warmup 10 --no-cpu-baseline
