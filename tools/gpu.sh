#!/bin/bash
# One parameterised runner for every GPU call (gpurun -- 'bash tools/gpu.sh RECIPE [RECIPE ...]').
# Each step has its own time limit; the first failing step ends the call (no GPU work after a fault, an
# abort or a timeout).  Logs: gpurun_out/<step>.log, summary: gpurun_out/status.log.
#
# Recipes (run in the order given):
#   check              pytest -m gpu (PYTEST_K / TESTS narrow it) + smoke
#   bench              the default bench line (python bench.py) → gpurun_out/bench.json
#   ab                 headline + planted lines of the in-tree library and of each LIBS variant
#                      (libstc_<n>.so); DTYPE=f32 for the fp32 kernels
#   configs            BASELINE configs 4 / 5 lines, fp64 + fp32, with the CPU baseline (DTYPES narrows)
#   c4ab / c5ab        config 4 / 5 A/B of the LIBS variants against the in-tree library (STEPS, WARMUP)
#   c2env/c4env/c5env  config 2 / 4 / 5 lines of the in-tree library under each ENVS="name:VAR=val,…" setting
#   feat               the featurisation line + its kernel profile + FETCH / WRITE passes
#   prof               rocprofv3 stats + PMC passes of WORKLOADS="name:bench args;…" (each into
#                      gpurun_out/prof_<name>; summarise with tools/pmc_summary.py --steady)
#   bitwise            tools/ab_bitwise.py: each LIBS variant's E-step / next() outputs vs the in-tree library's
#   counters           one --pmc pass of $COUNTERS (those this rocprofv3 lists) over the headline E-step
#   ubench             tools/ubench_f64 (the fp64 chain micro-benchmark)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
touch gpurun_out/status.log

step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "$(date +%T) start $name" >> gpurun_out/status.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$(date +%T) $name rc=$rc" >> gpurun_out/status.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
lib() { echo "spark-text-clustering_amd/stc/libstc_$1.so"; }
FAST="--no-cpu-baseline --no-secondary --no-hbm-copy"
PLANTED="--corpus zipf-lda --state planted"

r_check() {
  step pytest_gpu ${PYTEST_SECS:-900} python -u -m pytest ${TESTS:-tests} -x -v -m gpu --timeout 150 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"}
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
}
r_bench() {
  step bench ${BENCH_SECS:-600} python bench.py ${BENCH_ARGS:-}
  tail -n 1 gpurun_out/bench.log > gpurun_out/bench.json
}
r_ab() {
  local B="python bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-5} $FAST --dtype ${DTYPE:-f64}"
  step b_new 300 $B
  step p_new 300 $B $PLANTED
  for n in $LIBS; do
    step b_$n 300 env STC_LIB=$(lib $n) $B
    step p_$n 300 env STC_LIB=$(lib $n) $B $PLANTED
  done
}
r_configs() {
  local B="python bench.py --steps 20 --warmup 10 --no-secondary --no-hbm-copy"
  for c in 4 5; do
    for dt in ${DTYPES:-f64 f32}; do
      step c${c}_$dt 700 $B --config $c --dtype $dt $( [ "$dt" = f32 ] && echo --no-cpu-baseline )
      tail -n 1 gpurun_out/c${c}_$dt.log > gpurun_out/c${c}_$dt.json
    done
  done
}
r_bitwise() {
  for n in $LIBS; do step bw_$n 400 python tools/ab_bitwise.py spark-text-clustering_amd/stc/libstc.so $(lib $n); done
}
r_cab() {  # r_cab CONFIG
  local B="python bench.py --config $1 --steps ${STEPS:-6} --warmup ${WARMUP:-2} $FAST"
  for n in $LIBS; do step c$1_$n 500 env STC_LIB=$(lib $n) $B; done
  step c$1_new 500 $B
}
r_cenv() {  # r_cenv CONFIG: the in-tree library under each ENVS="name:VAR=val[,VAR=val] …" setting
  local B="python bench.py --config $1 --steps ${STEPS:-6} --warmup ${WARMUP:-2} $FAST"
  for spec in $ENVS; do step c$1_${spec%%:*} 500 env $(echo "${spec#*:}" | tr , ' ') $B; done
}
r_feat() {
  step feat 300 python bench.py --featurisation-only --steps 5
  rm -rf gpurun_out/featprof gpurun_out/featpmc
  local B="bench.py --featurisation-only --steps 3 --workers 1"
  step featprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/featprof -o fp --output-format csv -- python3 $B
  step featfetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/featpmc/fetch -o fetch --output-format csv -- python3 $B
  step featwrite 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/featpmc/write -o write --output-format csv -- python3 $B
}
prof_one() {  # prof_one NAME "bench args"
  local out=gpurun_out/prof_$1; rm -rf $out; mkdir -p $out
  # --workers 1: no corpus-generation worker processes forked after the profiler initialised the GPU
  local B="bench.py --steps ${STEPS:-5} --warmup ${WARMUP:-3} $FAST --workers 1 $2"
  for pass in ${PASSES:-stats fetch write sq}; do
    case $pass in
      stats) step $1_stats ${PROF_SECS:-400} rocprofv3 --kernel-trace --stats -d $out/stats -o stats --output-format csv -- python3 $B ;;
      fetch) step $1_fetch ${PROF_SECS:-400} rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o fetch --output-format csv -- python3 $B ;;
      write) step $1_write ${PROF_SECS:-400} rocprofv3 --pmc WRITE_SIZE -d $out/write -o write --output-format csv -- python3 $B ;;
      sq) step $1_sq ${PROF_SECS:-400} rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
            SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --kernel-include-regex "k_estep" -d $out/sq -o sq \
            --output-format csv -- python3 $B ;;
    esac
  done
}
r_prof() {
  local IFS_OLD=$IFS w
  IFS=';' read -ra WL <<< "${WORKLOADS:-headline_f64:}"
  IFS=$IFS_OLD
  for w in "${WL[@]}"; do prof_one "${w%%:*}" "${w#*:}"; done
}
r_counters() {
  local out=gpurun_out/counters; rm -rf $out; mkdir -p $out
  step counters_list 60 rocprofv3 -L
  local C
  C=$(python3 -c '
import re, sys
t = open("gpurun_out/counters_list.log").read()
print(" ".join(w for w in sys.argv[1].split() if re.search(r"\b%s\b" % re.escape(w.replace("_sum", "")), t)))' "$COUNTERS")
  [ -n "$C" ] || { echo "none of $COUNTERS listed" >> gpurun_out/status.log; return 0; }
  step counters 400 rocprofv3 --pmc $C --kernel-include-regex "${KREGEX:-k_estep}" -d $out/p -o p --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 $FAST --workers 1 ${BENCH_ARGS:-}
}
r_ubench() { step ubench 120 ./tools/ubench_f64; }

for r in "$@"; do
  case $r in
    check) r_check ;;
    bench) r_bench ;;
    ab) r_ab ;;
    bitwise) r_bitwise ;;
    configs) r_configs ;;
    c4ab) r_cab 4 ;;
    c5ab) r_cab 5 ;;
    c4env) r_cenv 4 ;;
    c5env) r_cenv 5 ;;
    c2env) r_cenv 2 ;;
    feat) r_feat ;;
    prof) r_prof ;;
    counters) r_counters ;;
    ubench) r_ubench ;;
    *) echo "unknown recipe $r" >> gpurun_out/status.log; exit 2 ;;
  esac
done
