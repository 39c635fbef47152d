#!/bin/bash
# config 4 fp64 at the BASELINE setting (20 timed after 10 warm-up): LIB variant vs the default, twice each, interleaved
mkdir -p gpurun_out; : > gpurun_out/status.log
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/status.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
L=spark-text-clustering_amd/stc/libstc_$LIB.so
B="python bench.py --config 4 --steps 20 --warmup 10 --no-cpu-baseline --no-secondary --no-hbm-copy"
step a1 400 env STC_LIB=$L $B
step b1 400 $B
step a2 400 env STC_LIB=$L $B
step b2 400 $B
