# Small-chain sweep tail check: the small-chain parity tests, then the
# reference call's bench leg and three single-chain calls.
# usage: gpu_lt.sh TAG
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=$1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs \
  -k "parallel_golden or last_customer or lane or newsim or chain_ids or sample_output or posterior or repair_shapes or underflow or table_limit" \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py --leg newsim_call > gpurun_out/${TAG}_newsim_call.json 2> gpurun_out/${TAG}_newsim_call.err || { tail -5 gpurun_out/${TAG}_newsim_call.err; exit 1; }
cat gpurun_out/${TAG}_newsim_call.json
for k in 1 2 3; do timeout -k 10 120 python3 scripts/newsim_once.py 10000 1 || exit 1; done
