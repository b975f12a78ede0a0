# Gauge recorder: GPU parity (every run_pair scenario compares gauge rows) and bench.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r29 && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -25 $O/pytest_gpu.log; exit 1; }
echo PYTEST_OK
A="--steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python bench.py $A > $O/default.json 2> $O/default.err || { echo B_FAILED; tail -5 $O/default.err; exit 1; }
echo BENCH_OK
timeout -k 10 120 python tools/bench_scan.py > $O/scan.json 2> $O/scan.err && echo SCAN_OK
