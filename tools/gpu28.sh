# Pruned (exact block-bound) scan vs full scan at C3.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r28 && mkdir -p $O
A="--steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python bench.py $A --pruned-scan > $O/pruned.json 2> $O/pruned.err || { echo P_FAILED; tail -5 $O/pruned.err; exit 1; }
echo DONE
