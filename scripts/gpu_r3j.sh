#!/bin/bash
# the whole GPU suite (configs[4] at full size and the full Reuters corpus included), then the repair shapes
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 \
    > gpurun_out/pytest_r3j.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_r3j.log; [ $rc -eq 0 ] || { echo "tests failed $rc"; tail -40 gpurun_out/pytest_r3j.log; exit 1; }
tail -25 gpurun_out/pytest_r3j.log
timeout -k 10 150 python -u scripts/r3_probe.py shapes > gpurun_out/r3j_shapes.log 2>&1 || { echo "shapes failed"; cat gpurun_out/r3j_shapes.log; exit 1; }
cat gpurun_out/r3j_shapes.log
