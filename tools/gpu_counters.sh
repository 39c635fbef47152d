#!/bin/bash
# One --pmc pass per model state (warm headline, planted) of the E-step kernels for the counters in
# $COUNTERS that this rocprofv3 knows (within one pass's hardware limits), time-limited; summarise
# with tools/counter_summary.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${CNT_OUT:-gpurun_out/counters}; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || exit $?
C=$(python3 - "$COUNTERS" <<'PY'
import re, sys
import os; t = open(os.environ.get("CNT_OUT", "gpurun_out/counters") + "/counters.txt").read()
print(" ".join(w for w in sys.argv[1].split() if re.search(r"\b%s\b" % re.escape(w.replace("_sum", "")), t)))
PY
)
echo "counters: $C" > $OUT/status.log
[ -n "$C" ] || exit 0
B="bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-hbm-copy --no-secondary --workers 1"
timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex k_estep -d $OUT/warm -o warm --output-format csv -- python3 $B > $OUT/warm.log 2>&1 &&
if [ -z "$NO_PLANTED" ]; then
timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex k_estep -d $OUT/planted -o planted --output-format csv -- python3 $B --corpus zipf-lda --state planted > $OUT/planted.log 2>&1
fi
