#!/bin/bash
# HEAD check after re-entry: full GPU suite, smoke, bench (all legs), rocprof kernel stats
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r3v.log 2>&1 \
    || { echo "tests failed"; tail -40 gpurun_out/pytest_r3v.log; exit 1; }
tail -2 gpurun_out/pytest_r3v.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || { echo "smoke failed"; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r3v.json 2> gpurun_out/bench_r3v.err \
    || { echo "bench failed $?"; tail -20 gpurun_out/bench_r3v.err; exit 1; }
cat gpurun_out/bench_r3v.json
echo done
