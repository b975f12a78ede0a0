# v5 hot loop (register source table, inline hot handlers): GPU parity + A/B (waves/EU) + profile.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r10
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r10/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; tail -15 gpurun_out/r10/pytest_gpu.log; exit 1; }
echo PYTEST_OK
A="--steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python bench.py $A > gpurun_out/r10/default.json 2> gpurun_out/r10/default.err || { echo B_FAILED; exit 1; }
for v in w3; do
  K10S_LIB=build/libk10s_$v.so timeout -k 10 300 python bench.py $A > gpurun_out/r10/$v.json 2> gpurun_out/r10/$v.err || { echo V_FAILED $v; exit 1; }
done
K10S_LIB=build/libk10s_prof.so timeout -k 10 300 python bench.py $A --profile > gpurun_out/r10/prof.json 2> gpurun_out/r10/prof.err || { echo P_FAILED; exit 1; }
echo DONE
