#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 240 python tools/diag_stat.py > gpurun_out/diag_stat.log 2>&1; echo "rc=$?" >> gpurun_out/diag_stat.log
