# Round 4: exact kernel v2 (ds_* instances, 1.3 KB Shared, log-det table, per-view
# marginal logs): parity, the New_Simulation probe, then the Reuters profile and
# the 8-chain trajectory continued (scripts/gpu_r4k.sh).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "exact or dropin or c_abi" \
  > gpurun_out/r4l_pytest.log 2>&1; rc=$?; tail -4 gpurun_out/r4l_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4l_smoke.log 2>&1 && tail -1 gpurun_out/r4l_smoke.log &&
for C in 1024 2048 4096; do timeout -k 10 200 python scripts/exact_probe.py $C >> gpurun_out/r4l_exact.json 2>> gpurun_out/r4l_exact.log || exit 1; done &&
MVC_EXACT_PROF=1 timeout -k 10 200 python scripts/exact_probe.py 2048 >> gpurun_out/r4l_exact.json 2>> gpurun_out/r4l_exact.log &&
cat gpurun_out/r4l_exact.json gpurun_out/r4l_exact.log &&
bash scripts/gpu_r4k.sh

