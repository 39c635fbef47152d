#!/bin/bash
# featurisation A/B: the bench line per library (LIBS: extra builds libstc_<n>.so) + a kernel profile of the default
mkdir -p gpurun_out; : > gpurun_out/status.log
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/status.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step t_feat 400 python -u -m pytest ${TESTS:-tests/test_gpu_feature.py} -x -v -m gpu --timeout 150 --timeout-method thread
step feat 300 python bench.py --featurisation-only --steps 5
for n in $LIBS; do step feat_$n 300 env STC_LIB=spark-text-clustering_amd/stc/libstc_$n.so python bench.py --featurisation-only --steps 5; done
[ -n "$NO_AB" ] || step feat_m0 300 env STC_TF_MODE=0 python bench.py --featurisation-only --steps 5
[ -n "$NO_AB" ] || step feat_nc 300 env STC_IDF_NO_CACHE=1 python bench.py --featurisation-only --steps 5
[ -n "$NO_AB" ] || step feat_d32 300 env STC_DF_U32=1 python bench.py --featurisation-only --steps 5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/featprof
step featprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/featprof -o fp --output-format csv -- python3 bench.py --featurisation-only --steps 3 --workers 1
if [ -n "$PROF2P" ]; then
  rm -rf gpurun_out/featprof2p
  STC_TF_MODE=0 step featprof2p 300 rocprofv3 --kernel-trace --stats -d gpurun_out/featprof2p -o fp --output-format csv -- python3 bench.py --featurisation-only --steps 3 --workers 1
fi
