#!/bin/bash
# grid E-step experiments: product bench, setprio build, stamps at 2 and 1 waves/SIMD
mkdir -p gpurun_out; : > gpurun_out/status.log
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/status.log
  if [ $rc -ge 124 ] || [ $rc -lt 0 ]; then exit $rc; fi
  return 0
}
B="bench.py --steps 10 --warmup 5 --no-cpu-baseline"
step bench_grid 240 python $B
STC_LIB=spark-text-clustering_amd/stc/libstc_prio.so step bench_prio 240 python $B
STC_LIB=spark-text-clustering_amd/stc/libstc_stamp.so step stamp_grid 240 python tools/stamp_estep.py
STC_GRID_LDS_PAD=80000 STC_LIB=spark-text-clustering_amd/stc/libstc_stamp.so step stamp_occ1 300 python tools/stamp_estep.py --steps 2
STC_GRID_LDS_PAD=80000 step bench_occ1 300 python $B
