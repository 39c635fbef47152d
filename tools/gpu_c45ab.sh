#!/bin/bash
# configs 4 and 5 E-step A/B of a variant library (LIB=<n>: libstc_<n>.so), with its wide/team parity tests
mkdir -p gpurun_out; : > gpurun_out/status.log
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/status.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
L=spark-text-clustering_amd/stc/libstc_$LIB.so
step t_wide 400 env STC_LIB=$L python -u -m pytest tests/test_gpu_lda.py tests/test_gpu_shapes.py -k "team or wide or config4 or config5" -x -v -m gpu --timeout 150 --timeout-method thread
B="python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-secondary --no-hbm-copy"
step c4_v 400 env STC_LIB=$L $B --config 4
step c4_b 400 $B --config 4
step c5_v 400 env STC_LIB=$L $B --config 5
step c5_b 400 $B --config 5
