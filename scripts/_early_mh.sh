#!/bin/bash
# A/B of the gated early MH (MVC_EARLY_MH), the GPU tests, and the north-star
# literal with many chains on one GPU (scripts/ns_chains.py).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_r2s.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_r2s.log; exit 1; }
tail -2 gpurun_out/pytest_r2s.log
for i in 1 2; do
  MVC_EARLY_MH=0 timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-extras --no-cpu-baseline \
      > gpurun_out/ab_off_$i.json 2>/dev/null || { echo "bench off failed"; exit 1; }
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-extras --no-cpu-baseline \
      > gpurun_out/ab_on_$i.json 2>/dev/null || { echo "bench on failed"; exit 1; }
  for f in gpurun_out/ab_off_$i.json gpurun_out/ab_on_$i.json; do
    python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['hbm']['pass_ms'])"
  done
done
timeout -k 10 300 python -u scripts/ns_chains.py 8 32 > gpurun_out/ns_chains.log 2>&1 || { echo "ns_chains failed"; tail -5 gpurun_out/ns_chains.log; exit 1; }
cat gpurun_out/ns_chains.log
