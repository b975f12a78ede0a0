# PMC passes (kernel-trace only, no sys/runtime traces) over one bench step.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pmc
R=$GRAFT_REPO_ROOT
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
SMALL="--replicas 4096 --pods 4096 --steps 1 --warmup 0 --no-cpu-baseline"
run() {  # name, bench args, counters...
  local name=$1; shift; local args=$1; shift
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pmc/$name -o run --pmc "$@" -- python3 $R/bench.py $args > $R/gpurun_out/pmc/$name.json 2> $R/gpurun_out/pmc/$name.err
}
run sq1 "$SMALL" SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS && echo SQ1_OK || exit 1
run sq2 "$SMALL" SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum && echo SQ2_OK || exit 1
run fetch "$SMALL" FETCH_SIZE && echo FETCH_OK || exit 1
run write "$SMALL" WRITE_SIZE && echo WRITE_OK || exit 1
run fetch_full "--steps 1 --warmup 0 --no-cpu-baseline" FETCH_SIZE && echo FETCHF_OK || exit 1
run write_full "--steps 1 --warmup 0 --no-cpu-baseline" WRITE_SIZE && echo WRITEF_OK
