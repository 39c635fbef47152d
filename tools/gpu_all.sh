#!/bin/bash
mkdir -p gpurun_out; : > gpurun_out/status.log
timeout -k 10 240 python tools/diag_wave.py > gpurun_out/diag_wave.log 2>&1; echo "diag rc=$?" >> gpurun_out/status.log
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/status.log
timeout -k 10 240 python bench.py --steps 10 --warmup 10 --no-cpu-baseline > gpurun_out/bench_wave.log 2>&1
rc=$?; echo "bench wave rc=$rc" >> gpurun_out/status.log; [ $rc -eq 0 ] || exit $rc
STC_DISABLE_WAVE=1 timeout -k 10 240 python bench.py --steps 10 --warmup 10 --no-cpu-baseline > gpurun_out/bench_v1.log 2>&1
echo "bench v1 rc=$?" >> gpurun_out/status.log
