# Parity on GPU + A/B: scan pipeline depth (p1/p2 default/p3), warm-handler inlining (s1), profiles.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r8
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r8/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; tail -15 gpurun_out/r8/pytest_gpu.log; exit 1; }
echo PYTEST_OK
A="--steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python bench.py $A > gpurun_out/r8/default.json 2> gpurun_out/r8/default.err || { echo B_FAILED; exit 1; }
for v in p1 p3 s1 s1_p1; do
  K10S_LIB=build/libk10s_$v.so timeout -k 10 300 python bench.py $A > gpurun_out/r8/$v.json 2> gpurun_out/r8/$v.err || { echo V_FAILED $v; exit 1; }
done
echo VAR_OK
for v in prof prof_s1; do
  K10S_LIB=build/libk10s_$v.so timeout -k 10 300 python bench.py $A --profile > gpurun_out/r8/$v.json 2> gpurun_out/r8/$v.err || { echo P_FAILED $v; exit 1; }
done
echo PROF_OK
