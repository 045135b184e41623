#!/bin/bash
# exact schedule with LDS-resident chain arrays: exact parity tests, then the New_Simulation shape probe
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_abi.py -x -v --timeout 300 --timeout-method thread \
    -k "exact or c_abi or smoke or async or golden or live_oracle or capacity or sweeps_per_launch" > gpurun_out/pytest_r3y.log 2>&1 \
    || { echo "tests failed"; grep -E "PASSED|FAILED|Error|error" gpurun_out/pytest_r3y.log | tail -30; exit 1; }
tail -2 gpurun_out/pytest_r3y.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || { echo "smoke failed"; exit 1; }
timeout -k 10 400 python -u scripts/newsim_probe.py > gpurun_out/newsim_r3y.json 2> gpurun_out/newsim_r3y.err \
    || { echo "probe failed"; tail gpurun_out/newsim_r3y.err; exit 1; }
cat gpurun_out/newsim_r3y.json

timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extras --steps 30 > gpurun_out/bench_r3y.json 2>/dev/null || { echo "bench failed"; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_r3y.json'));print('headline',d['value'],d['ms_per_step'],d['hbm']['pass_ms'])"
echo done
