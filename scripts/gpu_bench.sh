#!/bin/bash
# bench + rocprofv3 kernel-trace summary on one MI355X (round-1 measurement)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-r1}
timeout -k 10 900 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed $?"; exit 1; }
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
echo done
