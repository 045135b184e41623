#!/bin/bash
# round-3 HEAD: full GPU suite, smoke, bench (all legs), rocprof kernel stats of the headline
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r3ab.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/pytest_r3ab.log | tail -20; tail -3 gpurun_out/pytest_r3ab.log; exit 1; }
tail -1 gpurun_out/pytest_r3ab.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || { echo "smoke failed"; exit 1; }
timeout -k 10 700 python -u bench.py > gpurun_out/bench_r3ab.json 2> gpurun_out/bench_r3ab.err \
    || { echo "bench failed $?"; tail -20 gpurun_out/bench_r3ab.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/bench_r3ab.json'));print('headline',d['value'],d['ms_per_step'],d['hbm']['pass_ms'],d['roofline']['frac'],d['kernel_ms_per_sweep'])
e=d['extra']
for k in ('north_star_literal_gpu','north_star_literal_gpu_16chains','cold_start_gpu','configs1_gpu','exact_schedule_gpu'): print(k, json.dumps(e.get(k))[:300])
print('newsim', json.dumps(e.get('newsim_call'))[:1200])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3ab -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/prof_r3ab.log 2>&1 \
    || { echo "rocprof failed $?"; exit 1; }
head -6 gpurun_out/prof_r3ab/run_kernel_stats.csv
echo done
