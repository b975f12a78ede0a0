# SQ issue/wait breakdown of the v4 event-loop kernel (small config, one step per pass).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pmc9
R=$GRAFT_REPO_ROOT
SMALL="--replicas 4096 --pods 4096 --steps 1 --warmup 0 --no-cpu-baseline"
run() {
  local name=$1; shift
  cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pmc9/$name -o run --pmc "$@" -- python3 $R/bench.py $SMALL > $R/gpurun_out/pmc9/$name.json 2> $R/gpurun_out/pmc9/$name.err
}
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS && echo SQ1_OK || exit 1
run sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA && echo SQ2_OK || exit 1
run sq3 SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 && echo SQ3_OK
