# A/B of engine build variants on one MI355X + a kernel-trace profile of the default build.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
ARGS="--replicas 4096 --pods 4096 --steps 2 --warmup 1 --no-cpu-baseline"
for v in s0 s2 s3; do
  K10S_LIB=build/libk10s_$v.so timeout -k 10 240 python bench.py $ARGS > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err || exit 1
  echo "variant $v done"
done
timeout -k 10 120 python tools/bench_scan.py > gpurun_out/scan.json 2> gpurun_out/scan.err && echo SCAN_OK
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r01 -o bench -- python3 bench.py $ARGS > gpurun_out/prof_r01_bench.json 2> gpurun_out/prof_r01_bench.err && echo PROF_OK
