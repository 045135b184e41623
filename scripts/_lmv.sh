#!/bin/bash
# GPU tests with the producer-side view terms (A.lmv), A/B vs MVC_LMV=0, and
# the north-star literal with many chains under more hardware queues.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_r2t.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_r2t.log; exit 1; }
tail -2 gpurun_out/pytest_r2t.log
for i in 1 2; do
  MVC_LMV=0 timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-extras --no-cpu-baseline \
      > gpurun_out/lmv_off_$i.json 2>/dev/null || { echo "bench off failed"; exit 1; }
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-extras --no-cpu-baseline \
      > gpurun_out/lmv_on_$i.json 2>/dev/null || { echo "bench on failed"; exit 1; }
  for f in gpurun_out/lmv_off_$i.json gpurun_out/lmv_on_$i.json; do
    python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['hbm']['pass_ms'], d['kernel_ms_per_sweep'])"
  done
done
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python -u scripts/ns_chains.py 16 > gpurun_out/ns_chains_q16.log 2>&1 || { echo "ns_chains failed"; tail -5 gpurun_out/ns_chains_q16.log; exit 1; }
cat gpurun_out/ns_chains_q16.log
