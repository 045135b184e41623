#!/bin/bash
# exact sweeps-per-launch bisection; two-pass register draw (MVC_ZDRAW_TP=1) parity + A/B
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v --timeout 200 --timeout-method thread \
    -k "sweeps_per_launch or exact_golden" > gpurun_out/pytest_r3aa_exact.log 2>&1; echo "exact tests rc $?"
grep -E "PASSED|FAILED" gpurun_out/pytest_r3aa_exact.log
MVC_ZDRAW_TP=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "phase_a or zpath2 or config4_full or parallel_golden" > gpurun_out/pytest_r3aa_tp.log 2>&1 \
    || { echo "tp tests failed"; grep -E "PASSED|FAILED|Error" gpurun_out/pytest_r3aa_tp.log | tail -20; exit 1; }
tail -1 gpurun_out/pytest_r3aa_tp.log
for z in 1 0 1 0; do
  MVC_ZDRAW_TP=$z timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extras --steps 20 > gpurun_out/bench_r3aa_$z.json 2>/dev/null \
    || { echo "bench $z failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_r3aa_$z.json'));print('tp=$z',d['value'],d['hbm']['pass_ms'],d['kernel_ms_per_sweep'])"
done
echo done
