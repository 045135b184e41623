#!/bin/bash
# pipelined phase A: parity, then headline A/B (MVC_ZPIPE=1 / 0) and rocprof of the pipe
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
    -k "zpipe or zpath2 or golden or config4_full or warm_start or repair" > gpurun_out/pytest_r3w.log 2>&1 \
    || { echo "tests failed"; grep -E "PASSED|FAILED|Error|error" gpurun_out/pytest_r3w.log | tail -30; exit 1; }
tail -2 gpurun_out/pytest_r3w.log
for z in 3 0 1 2 3; do
  MVC_ZPIPE=$z timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extras --steps 20 > gpurun_out/bench_r3w_$z.json 2>gpurun_out/bench_r3w_$z.err \
    || { echo "bench $z failed"; tail gpurun_out/bench_r3w_$z.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_r3w_$z.json'));print('zpipe=$z',d['value'],d['hbm']['pass_ms'],d['kernel_ms_per_sweep'])"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3w -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/prof_r3w.log 2>&1 \
    || { echo "rocprof failed $?"; exit 1; }
find gpurun_out/prof_r3w -name "*kernel_stats.csv" | head -1 | xargs head -8
echo done
