# Heap pop with the min child's full entry fetched in the key batch: GPU parity, A/B vs HEAD, w6.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r30 && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -25 $O/pytest_gpu.log; exit 1; }
echo PYTEST_OK
A="--steps 2 --warmup 1 --no-cpu-baseline --no-scan-kernel"
timeout -k 10 300 python bench.py $A > $O/default.json 2> $O/default.err || { echo B_FAILED; tail -5 $O/default.err; exit 1; }
for v in head w6; do
  K10S_LIB=build/libk10s_$v.so timeout -k 10 300 python bench.py $A > $O/$v.json 2> $O/$v.err || { echo V_FAILED $v; tail -3 $O/$v.err; exit 1; }
done
timeout -k 10 300 python bench.py $A > $O/default2.json 2> $O/default2.err || { echo B2_FAILED; exit 1; }
echo DONE
