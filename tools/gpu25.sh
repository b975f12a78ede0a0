# Occupancy A/B after the scan changes: waves/SIMD 5 (default), 6, 7 and handler split 3.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r25 && mkdir -p $O
A="--steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python bench.py $A > $O/default.json 2> $O/default.err || { echo B_FAILED; tail -5 $O/default.err; exit 1; }
for v in w6 w6_s3 s3 w7_s3; do
  K10S_LIB=build/libk10s_$v.so timeout -k 10 300 python bench.py $A > $O/$v.json 2> $O/$v.err || { echo V_FAILED $v; tail -3 $O/$v.err; exit 1; }
done
echo DONE
