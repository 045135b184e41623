#!/bin/bash
# 16 / 32 concurrent literal chains, then the Reuters run (8 chains, cold start) with the reference's views
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/ns_chains.py 16 32 > gpurun_out/r3l_ns_chains.log 2>&1 || { echo "chains failed"; tail gpurun_out/r3l_ns_chains.log; exit 1; }
cat gpurun_out/r3l_ns_chains.log
timeout -k 10 800 python -u scripts/reuters_run.py --sweeps 200 --chains 8 --ari-every 5 --budget-s 620 \
    > gpurun_out/r3l_reuters.log 2>&1 || { echo "reuters failed"; tail gpurun_out/r3l_reuters.log; exit 1; }
tail -3 gpurun_out/r3l_reuters.log
