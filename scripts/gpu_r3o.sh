#!/bin/bash
# adaptive stay limit: parity subset, then configs[3] cold start and the repair shapes
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
    -k "repair or capacity or config2 or chains or golden or live_oracle or multichunk or warm_start or mfma_path or table_limit or config4" \
    > gpurun_out/pytest_r3o.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_r3o.log; exit 1; }
tail -2 gpurun_out/pytest_r3o.log
timeout -k 10 150 python3 -u scripts/coldstart.py --config c4 --sweeps 12 --budget-s 100 > gpurun_out/r3o_c4.log 2>&1 || { echo "c4 failed"; exit 1; }
tail -4 gpurun_out/r3o_c4.log
timeout -k 10 100 python3 -u scripts/r3_probe.py shapes > gpurun_out/r3o_shapes.log 2>&1 || { echo "shapes failed"; exit 1; }
cat gpurun_out/r3o_shapes.log
