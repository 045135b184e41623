# Round 5: eval grid sized by n, small chains batch 4 repair rounds --
# full GPU suite, the reference call, the newsim legs.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5al}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u scripts/newsim_prof.py > gpurun_out/${TAG}_newsim.log 2>&1 || exit 1
cat gpurun_out/${TAG}_newsim.log
timeout -k 10 300 python3 bench.py --leg newsim_call > gpurun_out/${TAG}_newsim_call.json 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_newsim_call.json | cut -c1-700
timeout -k 10 300 python3 bench.py --leg newsim_chains > gpurun_out/${TAG}_newsim_chains.json 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_newsim_chains.json | cut -c1-400
