# Round-1 evidence for the current kernel: GPU parity, default bench (with CPU baseline),
# rocprofv3 kernel stats of one bench step, PMC HBM-traffic passes (FETCH_SIZE / WRITE_SIZE).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/prof6 gpurun_out/pmc6
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu6.log 2>&1 || { echo "PYTEST FAILED"; tail -5 gpurun_out/pytest_gpu6.log; exit 1; }
echo PYTEST_OK
timeout -k 10 400 python bench.py > gpurun_out/bench6.json 2> gpurun_out/bench6.err || { echo BENCH_FAILED; tail -5 gpurun_out/bench6.err; exit 1; }
echo BENCH_OK
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof6 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/prof6/bench.json 2> $R/gpurun_out/prof6/bench.err || { echo PROF_FAILED; exit 1; }
echo PROF_OK
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pmc6/fetch -o run --pmc FETCH_SIZE -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc6/fetch.json 2> $R/gpurun_out/pmc6/fetch.err || { echo FETCH_FAILED; exit 1; }
echo FETCH_OK
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pmc6/write -o run --pmc WRITE_SIZE -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc6/write.json 2> $R/gpurun_out/pmc6/write.err || { echo WRITE_FAILED; exit 1; }
echo WRITE_OK
