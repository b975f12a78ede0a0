# GPU parity (incl. pruned-scan tests), pruned vs full scan, cycle attribution (K10S_PROF variant).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r7
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r7/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; tail -15 gpurun_out/r7/pytest_gpu.log; exit 1; }
echo PYTEST_OK
A="--steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python bench.py $A > gpurun_out/r7/pruned.json 2> gpurun_out/r7/pruned.err || { echo B1_FAILED; exit 1; }
timeout -k 10 300 python bench.py $A --full-scan > gpurun_out/r7/full.json 2> gpurun_out/r7/full.err || { echo B2_FAILED; exit 1; }
echo BENCH_OK
K10S_LIB=build/libk10s_prof.so timeout -k 10 300 python bench.py $A --profile > gpurun_out/r7/prof_pruned.json 2> gpurun_out/r7/prof_pruned.err || { echo P1_FAILED; exit 1; }
K10S_LIB=build/libk10s_prof.so timeout -k 10 300 python bench.py $A --profile --full-scan > gpurun_out/r7/prof_full.json 2> gpurun_out/r7/prof_full.err || { echo P2_FAILED; exit 1; }
K10S_LIB=build/libk10s_prof_w8.so timeout -k 10 300 python bench.py $A --profile --full-scan > gpurun_out/r7/prof_w8_full.json 2> gpurun_out/r7/prof_w8_full.err || { echo P3_FAILED; exit 1; }
echo PROF_OK
