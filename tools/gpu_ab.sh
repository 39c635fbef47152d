#!/bin/bash
# A/B of an E-step change: the LDA parity tests, the headline (and planted) bench lines with the new
# kernel (and, with OLD_LIB=path, with that earlier build of the library), then the stamp build's phase split
# (STAMP=1).  One time limit per step; stops at the first failure.
mkdir -p gpurun_out; : > gpurun_out/status.log
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/status.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
B="python bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-secondary --no-hbm-copy"
P="--corpus zipf-lda --state planted"
if [ "${TESTS:-default}" != "none" ]; then
  step t_lda ${T_SECS:-500} python -u -m pytest ${TESTS/default/tests/test_gpu_lda.py tests/test_gpu_shapes.py tests/test_gpu_config1.py} -x -v -m gpu --timeout 150 --timeout-method thread
fi
step b_new 240 $B
step p_new 240 $B $P
if [ -n "$OLD_LIB" ]; then  # a previous build of libstc.so, e.g. saved before an E-step change
  step b_old 240 env STC_LIB=$OLD_LIB $B
  step p_old 240 env STC_LIB=$OLD_LIB $B $P
fi
for lib in $LIBS; do  # experiment builds, e.g. LIBS="libstc_p1.so": headline (and planted) lines with each
  n=${lib%.so}; n=${n#libstc_}
  step b_$n 240 env STC_LIB=spark-text-clustering_amd/stc/$lib $B
  if [ -n "$LIBS_PLANTED" ]; then step p_$n 240 env STC_LIB=spark-text-clustering_amd/stc/$lib $B $P; fi
done
if [ -n "$CONFIGS" ]; then  # e.g. CONFIGS="5 4": the many-topic shapes' headline lines
  for c in $CONFIGS; do step c${c}_new 400 $B --config $c; done
fi
if [ -n "$STAMP" ]; then
  step stamp 200 env STC_LIB=spark-text-clustering_amd/stc/libstc_stamp.so python tools/stamp_rows64.py
  step stampp 200 env STC_LIB=spark-text-clustering_amd/stc/libstc_stamp.so python tools/stamp_rows64.py --corpus zipf-lda
fi
if [ -n "$PROF" ]; then  # rocprofv3 passes of the bench (PROF_PASSES, BENCH_ARGS, PROF_OUT as tools/gpu_prof.sh)
  step prof 900 bash tools/gpu_prof.sh
fi
if [ -n "$ICACHE" ]; then step icache 700 bash tools/gpu_icache.sh; fi
if [ -n "$COUNTERS" ]; then step counters 700 bash tools/gpu_counters.sh; fi
if [ -n "$EXIT_PROBE" ]; then  # last: the team-kernel exit under rocprofv3 (EXIT_ARGS="--close": explicit teardown)
  rm -rf gpurun_out/exitp
  step exitp 180 env TMPDIR=/tmp rocprofv3 --kernel-trace --stats -d gpurun_out/exitp -o exitp --output-format csv -- python3 tools/exit_probe.py gpurun_out/exitp_maps.txt $EXIT_ARGS
fi
