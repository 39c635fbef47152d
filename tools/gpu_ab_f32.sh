mkdir -p gpurun_out; : > gpurun_out/status.log
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/status.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="python bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-secondary --no-hbm-copy --dtype f32"
P="--corpus zipf-lda --state planted"
step t_all 600 python -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread
step f_new 240 $B
step fp_new 240 $B $P
step f_old 240 env STC_LIB=spark-text-clustering_amd/stc/libstc_old.so $B
step fp_old 240 env STC_LIB=spark-text-clustering_amd/stc/libstc_old.so $B $P
