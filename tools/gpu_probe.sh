#!/bin/bash
# One GPU call of diagnostics: the available PMC counters, the rows E-step stamp split (headline and
# planted), then (last, since it may end in the exit-time SIGSEGV under investigation) the team-kernel
# exit probe under rocprofv3.  EXIT_ARGS="--close" runs the probe with explicit teardown.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out; : > gpurun_out/status.log
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/status.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
if [ -n "$LIST" ]; then step counters 60 rocprofv3 -L; fi
if [ -n "$STAMP" ]; then
  step stamp 200 env STC_LIB=spark-text-clustering_amd/stc/libstc_stamp.so python tools/stamp_rows64.py
  step stampp 200 env STC_LIB=spark-text-clustering_amd/stc/libstc_stamp.so python tools/stamp_rows64.py --corpus zipf-lda
fi
if [ -n "$EXIT_PROBE" ]; then
  rm -rf gpurun_out/exitp
  step exitp 180 rocprofv3 --kernel-trace --stats -d gpurun_out/exitp -o exitp --output-format csv -- python3 tools/exit_probe.py gpurun_out/exitp_maps.txt $EXIT_ARGS
fi
