# Knob A/B on the v10 engine: FIFO window 16, no scan pipeline, handler split 1.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r32 && mkdir -p $O
A="--steps 2 --warmup 1 --no-cpu-baseline --no-scan-kernel"
timeout -k 10 300 python bench.py $A > $O/default.json 2> $O/default.err || { echo B_FAILED; tail -5 $O/default.err; exit 1; }
for v in q16 p0 s1; do
  K10S_LIB=build/libk10s_$v.so timeout -k 10 300 python bench.py $A > $O/$v.json 2> $O/$v.err || { echo V_FAILED $v; tail -3 $O/$v.err; exit 1; }
done
echo DONE
