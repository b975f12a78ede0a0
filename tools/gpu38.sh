# Streamed Alibaba CSV -> K10SPOD1 block through the GPU engine (tests/test_trace_soa.py), then the full GPU suite.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r38 && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -15 $O/pytest_gpu.log; exit 1; }
echo PYTEST_OK; grep -c PASSED $O/pytest_gpu.log; grep trace_soa $O/pytest_gpu.log; tail -1 $O/pytest_gpu.log
