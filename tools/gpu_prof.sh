#!/bin/bash
# rocprofv3 kernel stats + separate PMC passes (HBM traffic, SQ issue/wait) of the bench workload.
# Each step has its own time limit; the script stops at the first failure.
# PROF_PASSES="stats fetch write" limits the passes (default: all five).
# Summarise afterwards (here): python tools/pmc_summary.py gpurun_out/prof --tag rNN
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${PROF_OUT:-gpurun_out/prof}; rm -rf $OUT; mkdir -p $OUT
# --workers 1: no corpus-generation worker processes (forked after the profiler initialised the GPU,
# they hung a --pmc pass twice)
B="bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-hbm-copy --no-secondary --workers 1 ${BENCH_ARGS:-}"
PASSES=${PROF_PASSES:-"stats fetch write sq grbm"}
run() {  # run NAME SECONDS ARGS...
  local name=$1 secs=$2; shift 2
  case " $PASSES " in *" $name "*) ;; *) return 0 ;; esac
  timeout -k 10 "$secs" rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 $B > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc" >> $OUT/status.log; return $rc
}
run stats 300 --kernel-trace --stats &&
run fetch 300 --pmc FETCH_SIZE &&
run write 300 --pmc WRITE_SIZE &&
run sq 300 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --kernel-include-regex "k_estep" &&
run grbm 300 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "k_estep"
