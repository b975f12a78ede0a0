# Round-1 measurement of the committed engine: GPU parity, official bench (CPU baseline incl.),
# rocprofv3 kernel-trace stats, HBM PMC (FETCH/WRITE), TLB + L2 PMC, scan-only microbench.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r33 && mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -15 $O/pytest_gpu.log; exit 1; }
echo PYTEST_OK
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail -5 $O/bench.err; exit 1; }
echo BENCH_OK
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/prof.json 2> $R/$O/prof.err || { echo PROF_FAILED; exit 1; }
echo PROF_OK
run() { local name=$1; shift; cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $R/$O/$name -o run --pmc "$@" -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/$O/$name.json 2> $R/$O/$name.err; }
run fetch FETCH_SIZE && echo FETCH_OK || exit 1
run write WRITE_SIZE && echo WRITE_OK || exit 1
cd $R && K10S_LIB=build/libk10s_prof.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile > $R/$O/prof_cycles.json 2> $R/$O/prof_cycles.err && echo PCYC_OK
cd $R && timeout -k 10 120 python tools/bench_scan.py > $R/$O/scan.json 2> $R/$O/scan.err && echo SCAN_OK
