#!/bin/bash
# parity tests of the changed kernels, the featurisation line, and an E-step A/B (LIBS: extra builds)
mkdir -p gpurun_out; : > gpurun_out/status.log
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/status.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step t_par 700 python -u -m pytest ${TESTS:-tests/test_gpu_lda.py tests/test_gpu_shapes.py tests/test_gpu_tokenizer.py tests/test_gpu_feature.py} -x -v -m gpu --timeout 150 --timeout-method thread
step feat 300 python bench.py --featurisation-only --steps 5
B="python bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-secondary --no-hbm-copy"
P="--corpus zipf-lda --state planted"
step b_new 240 $B
step p_new 240 $B $P
for n in $LIBS; do
  step b_$n 240 env STC_LIB=spark-text-clustering_amd/stc/libstc_$n.so $B
  step p_$n 240 env STC_LIB=spark-text-clustering_amd/stc/libstc_$n.so $B $P
done
if [ -n "$FEAT_PROF" ]; then  # kernel-level split of the featurisation line
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  rm -rf gpurun_out/featprof
  step featprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/featprof -o fp --output-format csv -- python3 bench.py --featurisation-only --steps 3 --workers 1
fi
