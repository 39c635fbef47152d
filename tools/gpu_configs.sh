mkdir -p gpurun_out; : > gpurun_out/status.log
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/status.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="python bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-secondary --no-hbm-copy"
step c4 400 $B --config 4 &&
step c5 300 $B --config 5 &&
step c4f32 400 $B --config 4 --dtype f32 &&
step c5f32 300 $B --config 5 --dtype f32 &&
step profp 600 env PROF_PASSES="stats fetch write" BENCH_ARGS="--corpus zipf-lda --state planted" PROF_OUT=gpurun_out/profp bash tools/gpu_prof.sh &&
step prof5 400 env PROF_PASSES="stats" BENCH_ARGS="--config 5" PROF_OUT=gpurun_out/prof5 bash tools/gpu_prof.sh
