#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/r3_legs.py > gpurun_out/r3r_legs.log 2>&1 || { echo "legs failed"; tail gpurun_out/r3r_legs.log; exit 1; }
cat gpurun_out/r3r_legs.log
