# Round 5: small chains -- relabel inside the compaction block, no gated early MH --
# full GPU suite, the reference call, configs[1] cold, the literal.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5au}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u scripts/newsim_prof.py > gpurun_out/${TAG}_newsim.log 2>&1 || exit 1
head -1 gpurun_out/${TAG}_newsim.log
timeout -k 10 300 python3 bench.py --leg newsim_call > gpurun_out/${TAG}_newsim_call.json 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_newsim_call.json | cut -c1-300
timeout -k 10 200 python3 bench.py --leg cold_start_gpu > gpurun_out/${TAG}_cold.json 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_cold.json | cut -c100-300
timeout -k 10 200 python3 bench.py --leg north_star_literal_gpu > gpurun_out/${TAG}_lit.json 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_lit.json | cut -c80-200
