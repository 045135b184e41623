#!/bin/bash
# PMC passes over one warm north-star-literal sweep (the run kernel carries it):
# one counter group per rocprofv3 run, kernel-trace only.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-r3}
export TMPDIR=/tmp
run() {  # $1 = pass name, rest = counters
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmcr_${TAG}_$name -o run --output-format csv -- \
      python3 scripts/r3_probe.py ns1 > gpurun_out/pmcr_${TAG}_$name.log 2>&1 || { echo "pmc $name failed"; tail -5 gpurun_out/pmcr_${TAG}_$name.log; exit 1; }
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run b SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS SQ_IFETCH
run c SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC
python3 scripts/pmc_run_summary.py $TAG
