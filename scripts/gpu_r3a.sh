#!/bin/bash
# Round-3 first GPU call: full GPU tests, repair-state shapes, the
# New_Simulation.R call in both schedules, and SQ counters of the repair run
# kernel at the north-star literal (one warm sweep; kernel-trace + pmc only).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_r3a.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/pytest_r3a.log; exit 1; }
timeout -k 10 200 python -u scripts/r3_probe.py shapes > gpurun_out/r3a_shapes.log 2>&1 || { echo "shapes failed"; exit 1; }
timeout -k 10 200 python -u scripts/r3_probe.py newsim 2000 > gpurun_out/r3a_newsim.log 2>&1 || { echo "newsim failed"; exit 1; }
timeout -k 10 30 rocprofv3 -L > gpurun_out/r3a_counters.txt 2>&1 || true
pmc() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "seq_run" --pmc "$@" \
      -d gpurun_out/pmcrun_r3a_$name -o run --output-format csv -- \
      python3 scripts/r3_probe.py ns1 > gpurun_out/pmcrun_r3a_$name.log 2>&1 || { echo "pmc $name failed"; exit 1; }
}
pmc sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
pmc lds SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT
echo done
