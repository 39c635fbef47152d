#!/bin/bash
# Instruction-cache counters of the E-step at the warm and planted states: list the counters this
# rocprofv3 knows, keep the icache / ifetch ones, one --pmc pass per state (time-limited).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/icache; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || exit $?
C=$(python3 - <<'PY'
import re
t = open("gpurun_out/icache/counters.txt").read()
want = ["SQC_ICACHE_MISSES", "SQC_ICACHE_HITS", "SQ_IFETCH", "SQ_WAIT_INST_ANY"]
print(" ".join(w for w in want if re.search(r"\b%s\b" % w, t)))
PY
)
echo "counters: $C" > $OUT/status.log
[ -n "$C" ] || exit 0
B="bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-hbm-copy --no-secondary --workers 1"
timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex k_estep -d $OUT/warm -o warm --output-format csv -- python3 $B > $OUT/warm.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex k_estep -d $OUT/planted -o planted --output-format csv -- python3 $B --corpus zipf-lda --state planted > $OUT/planted.log 2>&1
