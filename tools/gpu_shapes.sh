#!/bin/bash
# E-step shape sweep for k=100 (STC_WAVE_SHAPE) — bench only; stops at the first crash/timeout.
mkdir -p gpurun_out; : > gpurun_out/status.log
for sh in 0 1 2; do
  STC_WAVE_SHAPE=$sh timeout -k 10 240 python bench.py --steps 10 --warmup 10 --no-cpu-baseline > gpurun_out/bench_shape$sh.log 2>&1
  rc=$?; echo "shape $sh rc=$rc" >> gpurun_out/status.log; [ $rc -eq 0 ] || exit $rc
done
