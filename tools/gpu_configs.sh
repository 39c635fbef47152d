#!/bin/bash
# BASELINE.md's config 4 / 5 rows: 20 timed minibatches after 10 warm-up, fp64 and fp32
mkdir -p gpurun_out; : > gpurun_out/status.log
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/status.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="python bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-secondary --no-hbm-copy"
step c4_f64 500 $B --config 4
step c4_f32 500 $B --config 4 --dtype f32
step c5_f64 400 $B --config 5
step c5_f32 400 $B --config 5 --dtype f32
