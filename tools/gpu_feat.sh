#!/bin/bash
# Featurisation A/B: the featurisation-only bench line with the current library and (OLD_LIB) an earlier
# build, then rocprofv3 kernel stats of the featurisation pass.  One time limit per step.
mkdir -p gpurun_out; : > gpurun_out/status.log
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/status.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step t_feat 300 python -u -m pytest tests/test_gpu_feature.py tests/test_gpu_tokenizer.py -x -q -m gpu --timeout 150 --timeout-method thread
step f_new 300 python bench.py --featurisation-only
if [ -n "$OLD_LIB" ]; then step f_old 300 env STC_LIB=$OLD_LIB python bench.py --featurisation-only; fi
step proff 400 env PROF_PASSES="stats" BENCH_ARGS="--featurisation-only" PROF_OUT=gpurun_out/proff bash tools/gpu_prof.sh
