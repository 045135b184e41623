#!/bin/bash
# The library's hardware-queue request for concurrent chains: the north-star
# literal with 16 chains, config 3 (Reuters, 8 chains) cold start, the chain
# tests and smoke.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/ns_chains.py 16 > gpurun_out/ns_chains_r2v.log 2>&1 || { echo "ns_chains failed"; tail -5 gpurun_out/ns_chains_r2v.log; exit 1; }
cat gpurun_out/ns_chains_r2v.log
timeout -k 10 200 python -u scripts/reuters_run.py --sweeps 3 --chains 8 --ari-every 1 --budget-s 120 > gpurun_out/reuters_r2v.log 2>&1 || { echo "reuters failed"; tail -5 gpurun_out/reuters_r2v.log; exit 1; }
tail -8 gpurun_out/reuters_r2v.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_reuters.py -x -v --timeout 250 --timeout-method thread -k "chains or reuters or lpall" > gpurun_out/pt_r2v.log 2>&1 || { tail -30 gpurun_out/pt_r2v.log; exit 1; }
tail -2 gpurun_out/pt_r2v.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
