# Concurrency sweep: same per-replica work, 1024..8192 replicas (1..2 waves per SIMD slot), cycle attribution.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r21 && mkdir -p $O
for R in 1024 2048 4096 5120 8192; do
  K10S_LIB=build/libk10s_prof.so timeout -k 10 300 python bench.py --replicas $R --steps 1 --warmup 1 --no-cpu-baseline --profile > $O/prof_$R.json 2> $O/prof_$R.err || { echo FAILED $R; exit 1; }
done
echo DONE
