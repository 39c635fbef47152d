#!/bin/bash
# config-4 / 5 E-step A/B: LIBS variants (libstc_<n>.so) on config 4, then the default on configs 4 and 5
mkdir -p gpurun_out; : > gpurun_out/status.log
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/status.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-secondary --no-hbm-copy"
for n in $LIBS; do step c4_$n 400 env STC_LIB=spark-text-clustering_amd/stc/libstc_$n.so $B --config 4; done
step c4_base 400 $B --config 4
[ -n "$C5" ] && step c5_base 400 $B --config 5
exit 0
