# Scan variants A/B (same box): HEAD build vs unconditional loads + SGPR pod request + f64 subtraction,
# branchy/branch-free node, 1/2-step load pipeline.  GPU parity on the default build first.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r24 && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -25 $O/pytest_gpu.log; exit 1; }
echo PYTEST_OK
A="--steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python bench.py $A > $O/default.json 2> $O/default.err || { echo B_FAILED; tail -5 $O/default.err; exit 1; }
for v in head bf0_p1 bf1_p1 bf1; do
  K10S_LIB=build/libk10s_$v.so timeout -k 10 300 python bench.py $A > $O/$v.json 2> $O/$v.err || { echo V_FAILED $v; tail -3 $O/$v.err; exit 1; }
done
echo DONE
