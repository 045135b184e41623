#!/bin/bash
# PMC passes on the z-resample kernel only (one counter group per run)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-r1}
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 600 rocprofv3 --kernel-trace --kernel-include-regex zresample --pmc "$@" -d gpurun_out/pmcz_${TAG}_$name -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcz_${TAG}_$name.log 2>&1 || { echo "pmc $name failed"; exit 1; }
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run b SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES
run c SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH
run d FETCH_SIZE
echo done
