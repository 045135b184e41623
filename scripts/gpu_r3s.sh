#!/bin/bash
# how often the repair's decision equals phase A's (prof build), and the bench's child legs
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
MVC_HIP_LIB=$GRAFT_REPO_ROOT/build_variants/prof/libmvc_hip.so timeout -k 10 200 python -u scripts/r3_probe.py shapes \
    > gpurun_out/r3s_prof.log 2>&1 || { echo "prof failed"; tail gpurun_out/r3s_prof.log; exit 1; }
grep runprof gpurun_out/r3s_prof.log
timeout -k 10 300 python3 -u bench.py --leg ns16 > gpurun_out/r3s_leg.log 2>&1 || { echo "leg failed"; tail gpurun_out/r3s_leg.log; exit 1; }
cat gpurun_out/r3s_leg.log
