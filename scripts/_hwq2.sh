#!/bin/bash
# Hardware queues requested by the Python loader: the headline bench (must not
# change), the north-star literal with 16 chains, config 3 with 8 chains.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r2w.json 2> gpurun_out/bench_r2w.err || { echo "bench failed"; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_r2w.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['hbm']['pass_ms'], d['extra']['north_star_literal_gpu'])"
timeout -k 10 200 python -u scripts/ns_chains.py 16 > gpurun_out/ns_chains_r2w.log 2>&1 || { echo "ns_chains failed"; tail -5 gpurun_out/ns_chains_r2w.log; exit 1; }
cat gpurun_out/ns_chains_r2w.log
timeout -k 10 200 python -u scripts/reuters_run.py --sweeps 3 --chains 8 --ari-every 1 --budget-s 120 > gpurun_out/reuters_r2w.log 2>&1 || { echo "reuters failed"; tail -5 gpurun_out/reuters_r2w.log; exit 1; }
tail -3 gpurun_out/reuters_r2w.log
