#!/bin/bash
# diagnose the serial multi-chain fault: the test alone (kernels serialised), then the whole GPU suite in the new order
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r3ae.log 2>&1; rc=$?
echo "suite rc $rc"; grep -E "FAILED|Error" gpurun_out/pytest_r3ae.log | head -8; tail -1 gpurun_out/pytest_r3ae.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || { echo "smoke failed"; exit 1; }
timeout -k 10 700 python -u bench.py > gpurun_out/bench_r3ae.json 2> gpurun_out/bench_r3ae.err || { echo "bench failed"; tail gpurun_out/bench_r3ae.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_r3ae.json'));print('headline',d['value'],d['ms_per_step'],d['roofline']['frac'])"
echo done
