# Round 4: mvc_run's sample emission split over host threads: the tests
# through mvc_run, then the New_Simulation chains leg.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_posterior.py -x -v --timeout 300 --timeout-method thread \
  -k "exact or dropin or c_abi or run_ or golden or posterior" > gpurun_out/r4mt_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r4mt_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --leg newsim_chains > gpurun_out/r4mt_newsim_chains.json 2> gpurun_out/r4mt.log && cat gpurun_out/r4mt_newsim_chains.json
