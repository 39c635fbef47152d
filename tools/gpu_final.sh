#!/bin/bash
# round-close check: the GPU suite, smoke, the default bench line, the featurisation kernel profile
mkdir -p gpurun_out; : > gpurun_out/status.log
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/status.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/featprof
step featprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/featprof -o fp --output-format csv -- python3 bench.py --featurisation-only --steps 3 --workers 1
