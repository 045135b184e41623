#!/bin/bash
# bench (all legs) + rocprofv3 kernel-trace summary of the headline
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r3p.json 2> gpurun_out/bench_r3p.err \
    || { echo "bench failed $?"; tail -20 gpurun_out/bench_r3p.err; exit 1; }
cat gpurun_out/bench_r3p.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3p -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/prof_r3p.log 2>&1 \
    || { echo "rocprof failed $?"; exit 1; }
echo done
