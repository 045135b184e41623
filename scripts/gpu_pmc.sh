#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-r1}
export TMPDIR=/tmp
run() {  # $1 = pass name, rest = counters
  local name=$1; shift
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc_${TAG}_$name -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_${TAG}_$name.log 2>&1 || { echo "pmc $name failed"; exit 1; }
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
echo done
