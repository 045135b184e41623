# ChainSet lane_batch check: the chain tests, then the reference call with
# 16 chains (scripts/newsim_once.py) and the bench's newsim legs.
# usage: gpu_lb.sh TAG
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=$1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs \
  -k "chains or lane_batch or chain_ids or logical or sample_output or posterior or last_customer or parallel_golden" \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
for C in 16 4 1; do timeout -k 10 120 python3 scripts/newsim_once.py 3000 $C || exit 1; done
timeout -k 10 400 python -u bench.py --leg newsim_chains > gpurun_out/${TAG}_newsim_chains.json 2> gpurun_out/${TAG}_newsim_chains.err || { tail -5 gpurun_out/${TAG}_newsim_chains.err; exit 1; }
cat gpurun_out/${TAG}_newsim_chains.json
