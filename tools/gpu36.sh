# Scan without filtered[0] tracking when no score can be NaN (weight 1, both requests > 0):
# GPU parity, A/B vs HEAD on one box, then the official measurement sequence of tools/gpu22.sh.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r36 && mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -15 $O/pytest_gpu.log; exit 1; }
echo PYTEST_OK
A="--steps 2 --warmup 1 --no-cpu-baseline --no-scan-kernel"
timeout -k 10 300 python bench.py $A > $O/ab_new.json 2> $O/ab_new.err || { echo AB_FAILED; exit 1; }
K10S_LIB=build/libk10s_head.so timeout -k 10 300 python bench.py $A > $O/ab_head.json 2> $O/ab_head.err || { echo AB_FAILED; exit 1; }
timeout -k 10 300 python bench.py $A > $O/ab_new2.json 2> $O/ab_new2.err || { echo AB_FAILED; exit 1; }
echo AB_OK
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail -5 $O/bench.err; exit 1; }
echo BENCH_OK
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/prof.json 2> $R/$O/prof.err || { echo PROF_FAILED; exit 1; }
echo PROF_OK
run() { local name=$1; shift; cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $R/$O/$name -o run --pmc "$@" -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/$O/$name.json 2> $R/$O/$name.err; }
run fetch FETCH_SIZE && echo FETCH_OK || exit 1
run write WRITE_SIZE && echo WRITE_OK || exit 1
cd $R && K10S_LIB=build/libk10s_prof.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile > $R/$O/prof_cycles.json 2> $R/$O/prof_cycles.err && echo PCYC_OK
