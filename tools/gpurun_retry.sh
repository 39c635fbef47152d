#!/bin/bash
# Run one gpurun call; retry ONLY when the box failed on the infrastructure side before our
# command started (status "transient" / exit 3).  A failure of our own command is never retried.
cmd="$1"; to="${2:-1200}"
for attempt in 1 2 3 4 5 6; do
  rm -f gpurun_out/.last_call.json
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$rc" = "3" ] || [ "$st" = "transient" ]; then
    echo "[retry] infrastructure transient (rc=$rc status=$st); sleeping 60s"; sleep 60; continue
  fi
  exit $rc
done
exit 3
