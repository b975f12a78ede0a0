# v6 A/B of semantics-neutral build knobs: handler inlining (K10S_SPLIT 0/1/2) and occupancy (waves/EU 4/5).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r18 && mkdir -p $O
A="--steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python bench.py $A > $O/default.json 2> $O/default.err || { echo B_FAILED; tail -5 $O/default.err; exit 1; }
for v in w4 w4_p2 w5_p2; do
  K10S_LIB=build/libk10s_$v.so timeout -k 10 300 python bench.py $A > $O/$v.json 2> $O/$v.err || { echo V_FAILED $v; tail -3 $O/$v.err; exit 1; }
done
echo DONE
