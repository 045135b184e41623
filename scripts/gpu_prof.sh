#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-r1}
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
echo done
