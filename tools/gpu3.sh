# Parity on the GPU, then A/B of inlining variants, then the default bench and its rocprofv3 summary.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; exit 1; }
echo SMOKE_OK
ARGS="--replicas 4096 --pods 4096 --steps 2 --warmup 1 --no-cpu-baseline"
for v in s0 s1 s3; do
  K10S_LIB=build/libk10s_$v.so timeout -k 10 240 python bench.py $ARGS > gpurun_out/var3_$v.json 2> gpurun_out/var3_$v.err || exit 1
done
timeout -k 10 240 python bench.py $ARGS > gpurun_out/var3_default.json 2> gpurun_out/var3_default.err || exit 1
echo VARIANTS_OK
timeout -k 10 500 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
echo BENCH_OK
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof3_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof3_bench.err && echo PROF_OK
