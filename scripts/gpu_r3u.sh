#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/r3_vpdebug.py > gpurun_out/r3u_vpdebug.log 2>&1; echo "rc $?"
grep -v "^mvc vp" gpurun_out/r3u_vpdebug.log | tail -20; grep "^mvc vp" gpurun_out/r3u_vpdebug.log | head -12
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v --timeout 200 --timeout-method thread -k "value_prediction or d16" > gpurun_out/pytest_r3u.log 2>&1; echo "pytest rc $?"
grep -E "PASSED|FAILED" gpurun_out/pytest_r3u.log
