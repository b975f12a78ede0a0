# PMC: LDS bank conflicts, wave residency and L2 hit rate of k10s_run_kernel (final round-1 build).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r34 && mkdir -p $O
R=$GRAFT_REPO_ROOT
run() { local name=$1; shift; cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $R/$O/$name -o run --pmc "$@" -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-scan-kernel > $R/$O/$name.json 2> $R/$O/$name.err; }
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE && echo LDS_OK || exit 1
run l2 TCC_HIT_sum TCC_MISS_sum SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU && echo L2_OK
