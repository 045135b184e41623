#!/bin/bash
# PMC passes over the reference's own call (N = 200, V = 5, 300 sweeps; the
# small chains' lane loop, mvc_seq_run_kernel<5>): one counter group per
# rocprofv3 run, kernel-trace only; summary over the run kernel's launches.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-r6}
export TMPDIR=/tmp
run() {  # $1 = pass name, rest = counters
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmcr_${TAG}_$name -o run --output-format csv -- \
      python3 scripts/newsim_once.py 1300 > gpurun_out/pmcr_${TAG}_$name.log 2>&1 || { echo "pmc $name failed"; tail -5 gpurun_out/pmcr_${TAG}_$name.log; exit 1; }
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run b SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS SQ_IFETCH
run c SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ
python3 scripts/pmc_run_summary.py $TAG
