#!/bin/bash
# several workloads' tools/gpu_prof.sh passes in one call: WORKLOADS="name:bench args;name:bench args"
# (each into gpurun_out/prof_<name>); stops at the first failing pass
IFS=';' read -ra WL <<< "$WORKLOADS"
for w in "${WL[@]}"; do
  name=${w%%:*}; args=${w#*:}
  echo "== $name: $args" >> gpurun_out/prof_multi.log
  PROF_OUT=gpurun_out/prof_$name BENCH_ARGS="$args" bash tools/gpu_prof.sh || { echo "$name failed" >> gpurun_out/prof_multi.log; exit 1; }
  echo "$name ok" >> gpurun_out/prof_multi.log
done
