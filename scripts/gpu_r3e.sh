#!/bin/bash
# run kernel phase profile (LDS tick counters) + the wave-per-customer path for comparison
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
MVC_HIP_LIB=$GRAFT_REPO_ROOT/build_variants/prof/libmvc_hip.so timeout -k 10 200 python -u scripts/r3_probe.py shapes \
    > gpurun_out/r3e_prof.log 2>&1 || { echo "prof failed"; tail gpurun_out/r3e_prof.log; exit 1; }
grep -E "runprof|tag" gpurun_out/r3e_prof.log
MVC_LC=0 timeout -k 10 200 python -u scripts/r3_probe.py shapes > gpurun_out/r3e_lc0.log 2>&1 || { echo "lc0 failed"; tail gpurun_out/r3e_lc0.log; exit 1; }
echo "MVC_LC=0:"; cat gpurun_out/r3e_lc0.log
