# Round 5: chain-batched repair -- multi-chain parity, then the literal with
# 16 and 64 chains at HIP's default 4 hardware queues, and the reference's
# call with 16 chains.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp GPU_MAX_HW_QUEUES=4
TAG=${1:-r5o}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_posterior.py -x -v --timeout 300 --timeout-method thread \
  -k "chains or last_customer or n_devices or pooled or async_sample or posterior or capacity" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u scripts/ns_chains.py 16 64 > gpurun_out/${TAG}_ns_chains.log 2>&1 || { tail -3 gpurun_out/${TAG}_ns_chains.log; exit 1; }
cat gpurun_out/${TAG}_ns_chains.log
timeout -k 10 300 python3 bench.py --leg newsim_chains > gpurun_out/${TAG}_newsim_chains.json 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_newsim_chains.json | cut -c1-500
