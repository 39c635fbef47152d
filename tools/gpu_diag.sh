#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 240 python tools/diag_wave.py > gpurun_out/diag_wave.log 2>&1; echo "diag rc=$?" >> gpurun_out/diag_wave.log
