# v6: delay-class FIFO windows + heap top levels in LDS. GPU parity, bench, FQW A/B, cycle attribution.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r20 && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -15 $O/pytest_gpu.log; exit 1; }
echo PYTEST_OK
A="--steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python bench.py $A > $O/default.json 2> $O/default.err || { echo B_FAILED; tail -5 $O/default.err; exit 1; }
echo BENCH_OK
for v in; do
  K10S_LIB=build/libk10s_$v.so timeout -k 10 300 python bench.py $A > $O/$v.json 2> $O/$v.err || { echo V_FAILED $v; exit 1; }
done
echo VAR_OK
K10S_LIB=build/libk10s_prof.so timeout -k 10 300 python bench.py $A --profile > $O/prof.json 2> $O/prof.err || { echo P_FAILED; exit 1; }
echo DONE
