#!/bin/bash
# single-asm Horner exp: bitwise tests, phase A alone, parity subset; full bench; rocprof of the headline
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "exp_log or phase_a or zpath2 or golden or config4_full or warm_start or repair or live_oracle or chains" > gpurun_out/pytest_r3x.log 2>&1 \
    || { echo "tests failed"; grep -E "PASSED|FAILED|Error|error" gpurun_out/pytest_r3x.log | tail -30; exit 1; }
tail -2 gpurun_out/pytest_r3x.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r3x.json 2> gpurun_out/bench_r3x.err \
    || { echo "bench failed $?"; tail -20 gpurun_out/bench_r3x.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/bench_r3x.json'));print(d['value'],d['hbm']['pass_ms'],d['kernel_ms_per_sweep'])
e=d['extra']
for k in ('north_star_literal_gpu','north_star_literal_gpu_16chains','cold_start_gpu'): print(k, json.dumps(e.get(k))[:400])
print('newsim', json.dumps(e.get('newsim_call'))[:900])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3x -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/prof_r3x.log 2>&1 \
    || { echo "rocprof failed $?"; exit 1; }
find gpurun_out/prof_r3x -name "*kernel_stats.csv" | head -1 | xargs head -6
echo done
