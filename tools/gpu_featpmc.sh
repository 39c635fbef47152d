#!/bin/bash
# featurisation PMC passes (HBM traffic per kernel): FETCH_SIZE and WRITE_SIZE in separate runs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/featpmc; rm -rf $OUT; mkdir -p $OUT
B="bench.py --featurisation-only --steps 3 --workers 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 $B > $OUT/fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 $B > $OUT/write.log 2>&1
