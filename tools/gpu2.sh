cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; echo "PYTEST rc=$?"
K10S_LIB=build/libk10s_s1.so timeout -k 10 300 python -m pytest tests -m gpu -q -k "fuzz_gpu or reference" > gpurun_out/pytest_gpu_s1.log 2>&1; echo "PYTEST_S1 rc=$?"
ARGS="--replicas 4096 --pods 4096 --steps 2 --warmup 1 --no-cpu-baseline"
for v in s0 s3; do
  K10S_LIB=build/libk10s_$v.so timeout -k 10 240 python bench.py $ARGS > gpurun_out/var2_$v.json 2> gpurun_out/var2_$v.err || exit 1
done
timeout -k 10 240 python bench.py $ARGS > gpurun_out/var2_default.json 2> gpurun_out/var2_default.err || exit 1
timeout -k 10 120 python tools/bench_scan.py > gpurun_out/scan2.json 2> gpurun_out/scan2.err && echo SCAN_OK
