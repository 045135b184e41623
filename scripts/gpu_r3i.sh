#!/bin/bash
# lane-column loop: register cursor, two barriers per step, births in their own kernel
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
    -k "repair or capacity or config2 or chains or golden or live_oracle or multichunk or warm_start or mfma_path or table_limit" \
    > gpurun_out/pytest_r3i.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_r3i.log; exit 1; }
tail -2 gpurun_out/pytest_r3i.log
timeout -k 10 200 python -u scripts/r3_probe.py shapes > gpurun_out/r3i_shapes.log 2>&1 || { echo "shapes failed"; cat gpurun_out/r3i_shapes.log; exit 1; }
cat gpurun_out/r3i_shapes.log
MVC_HIP_LIB=$GRAFT_REPO_ROOT/build_variants/prof/libmvc_hip.so timeout -k 10 200 python -u scripts/r3_probe.py shapes \
    > gpurun_out/r3i_prof.log 2>&1 || { echo "prof failed"; tail gpurun_out/r3i_prof.log; exit 1; }
grep runprof gpurun_out/r3i_prof.log
