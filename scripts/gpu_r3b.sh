#!/bin/bash
# lane-column repair evaluation: parity tests of the repair paths, then the
# state shapes where the repair carries the sweep (timings)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
    -k "repair or capacity or config2 or chains or golden or live_oracle or multichunk or warm_start or mfma_path" \
    > gpurun_out/pytest_r3b.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_r3b.log; exit 1; }
tail -3 gpurun_out/pytest_r3b.log
timeout -k 10 200 python -u scripts/r3_probe.py shapes > gpurun_out/r3b_shapes.log 2>&1 || { echo "shapes failed"; cat gpurun_out/r3b_shapes.log; exit 1; }
cat gpurun_out/r3b_shapes.log
echo done
