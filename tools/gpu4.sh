# Parity on the GPU, A/B of build variants, default bench.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK
ARGS="--replicas 4096 --pods 4096 --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 240 python bench.py $ARGS > gpurun_out/var4_default.json 2> gpurun_out/var4_default.err || exit 1
for v in s0 s3 w4 s3w4; do
  K10S_LIB=build/libk10s_$v.so timeout -k 10 240 python bench.py $ARGS > gpurun_out/var4_$v.json 2> gpurun_out/var4_$v.err || exit 1
done
echo VARIANTS_OK
timeout -k 10 500 python bench.py --no-cpu-baseline > gpurun_out/bench4_default.json 2> gpurun_out/bench4_default.err && echo BENCH_OK
