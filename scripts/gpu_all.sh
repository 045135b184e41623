#!/bin/bash
# parity tests then bench + rocprof; stops at the first failure
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-r1}
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout=300 -rf > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || { echo "tests failed"; exit 1; }
bash scripts/gpu_bench.sh $TAG
