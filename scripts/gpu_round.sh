#!/bin/bash
# GPU parity tests, then bench + rocprofv3 kernel-trace summary; stops at the
# first failure.  Usage: bash scripts/gpu_round.sh TAG [pytest -k expr]
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-r2}
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" \
      > gpurun_out/pytest_$TAG.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > gpurun_out/pytest_$TAG.log 2>&1
fi
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || { echo "tests failed $rc"; exit 1; }
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
    || { echo "bench failed $?"; exit 1; }
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/prof_$TAG.log 2>&1 \
    || { echo "rocprof failed $?"; exit 1; }
echo done
