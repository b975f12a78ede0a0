cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK
ARGS="--replicas 4096 --pods 4096 --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 240 python bench.py $ARGS > gpurun_out/var5_default.json 2> gpurun_out/var5_default.err || exit 1
for v in s3 w0 w5; do
  K10S_LIB=build/libk10s_$v.so timeout -k 10 240 python bench.py $ARGS > gpurun_out/var5_$v.json 2> gpurun_out/var5_$v.err || exit 1
done
echo VARIANTS_OK
timeout -k 10 500 python bench.py --no-cpu-baseline > gpurun_out/bench5_default.json 2> gpurun_out/bench5_default.err && echo BENCH_OK
