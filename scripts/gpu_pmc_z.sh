#!/bin/bash
# PMC passes on the z-resample pass kernels (lp producer + draw), one counter
# group per rocprofv3 run (kernel-trace only), then a traffic summary.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-r1}
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 600 rocprofv3 --kernel-trace --kernel-include-regex "lpview|lpall|lpgen|zdraw|zfused" --pmc "$@" \
      -d gpurun_out/pmcz_${TAG}_$name -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/pmcz_${TAG}_$name.log 2>&1 || { echo "pmc $name failed"; exit 1; }
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS
python3 scripts/pmc_summary.py $TAG > gpurun_out/pmc_traffic_$TAG.json || exit 1
echo done
