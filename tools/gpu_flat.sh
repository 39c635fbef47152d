#!/bin/bash
# scratch (FLAT-segment) instructions per wave of the headline E-step: are the spills in the fixed-point loop?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/flat; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_FLAT SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "k_estep_rows64" -d $OUT/p -o p --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-hbm-copy --no-secondary --workers 1 > $OUT/p.log 2>&1
