#!/bin/bash
# config-4 fp64 team size A/B (STC_WIDE_TEAM forces P)
mkdir -p gpurun_out; : > gpurun_out/status.log
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/status.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="python bench.py --config 4 --steps 6 --warmup 2 --no-cpu-baseline --no-secondary --no-hbm-copy"
for p in ${PS:-5 6}; do step c4_p$p 400 env STC_WIDE_TEAM=$p $B; done
step c4_p0 400 $B
