#!/bin/bash
mkdir -p gpurun_out
STC_LIB=spark-text-clustering_amd/stc/libstc_stamp.so timeout -k 10 300 python tools/stamp_estep.py > gpurun_out/stamp.log 2>&1 || exit $?
for sh in 1 2 3; do
  STC_WAVE_SHAPE=$sh timeout -k 10 200 python bench.py --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/shape$sh.log 2>&1 || exit $?
done
