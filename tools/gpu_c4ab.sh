#!/bin/bash
# config-4 E-step A/B of the granule store policy: team parity tests on the variant, then both bench lines
mkdir -p gpurun_out; : > gpurun_out/status.log
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/status.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step t_team 400 env STC_LIB=spark-text-clustering_amd/stc/libstc_GP.so python -u -m pytest tests/test_gpu_lda.py -k "team or wide" -x -v -m gpu --timeout 150 --timeout-method thread
B="python bench.py --config 4 --steps 6 --warmup 2 --no-cpu-baseline --no-secondary --no-hbm-copy"
step c4_gp 400 env STC_LIB=spark-text-clustering_amd/stc/libstc_GP.so $B
step c4_base 400 $B
