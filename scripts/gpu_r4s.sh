# Round 4: exact kernel at HEAD: parity, the probe, and its PMC passes.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "exact or dropin or c_abi" \
  > gpurun_out/r4s_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r4s_pytest.log; [ $rc -eq 0 ] || exit 1
for C in 2048 4096; do timeout -k 10 200 python scripts/exact_probe.py $C >> gpurun_out/r4s_exact.json 2>> gpurun_out/r4s_exact.log || exit 1; done
cat gpurun_out/r4s_exact.json
bash scripts/gpu_pmc_exact.sh r4s > gpurun_out/r4s_pmc_exact.json 2> gpurun_out/r4s_pmc_exact.err; cat gpurun_out/r4s_pmc_exact.json
