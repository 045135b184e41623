#!/bin/bash
# value prediction: parity (new test + the repair / golden subset), then the shapes' timings and vp stats
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
    -k "value_prediction or repair or capacity or config2 or chains or golden or live_oracle or multichunk or warm_start or mfma_path or table_limit" \
    > gpurun_out/pytest_r3t.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest_r3t.log; exit 1; }
tail -2 gpurun_out/pytest_r3t.log
MVC_VP_STATS=1 timeout -k 10 150 python3 -u scripts/r3_probe.py shapes > gpurun_out/r3t_shapes.log 2>&1 || { echo "shapes failed"; tail gpurun_out/r3t_shapes.log; exit 1; }
cat gpurun_out/r3t_shapes.log
