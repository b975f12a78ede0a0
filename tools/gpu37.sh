# Re-entry confirmation on a fresh box: the in-tree .so rebuilt in a re-created container,
# GPU parity suite, smoke(), then the default bench line (the driver's own round-end sequence).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r37 && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -15 $O/pytest_gpu.log; exit 1; }
echo PYTEST_OK; tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -15 $O/smoke.log; exit 1; }
echo SMOKE_OK
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail -5 $O/bench.err; exit 1; }
echo BENCH_OK; cat $O/bench.json
