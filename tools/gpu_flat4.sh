#!/bin/bash
# scratch (FLAT-segment) instructions per wave of the config-4 team E-step
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/flat4; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_FLAT SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "k_estep_wide" -d $OUT/p -o p --output-format csv -- python3 bench.py --config 4 --steps 2 --warmup 1 --state-minibatches 5 --no-cpu-baseline --no-hbm-copy --no-secondary --workers 1 > $OUT/p.log 2>&1
