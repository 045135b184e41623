#!/bin/bash
# parity tests, z-kernel breakdown, bench (no rocprof)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-r1}
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout=300 -rf > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || { echo "tests failed"; exit 1; }
timeout -k 10 600 python scripts/zbreak.py 0 > gpurun_out/zbreak_$TAG.txt 2>&1 || { echo "zbreak failed"; exit 1; }
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; exit 1; }
echo done
