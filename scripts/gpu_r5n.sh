# Round 5: births committed inside the lane-column run kernels, no grid
# windows for small chains: full GPU suite, the reference's call, the literal.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5n}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u scripts/newsim_prof.py > gpurun_out/${TAG}_newsim.log 2>&1 || exit 1
MVC_SMALL_N=0 timeout -k 10 120 python -u scripts/newsim_prof.py >> gpurun_out/${TAG}_newsim.log 2>&1 || exit 1
cat gpurun_out/${TAG}_newsim.log
timeout -k 10 300 python3 bench.py --leg north_star_literal_gpu > gpurun_out/${TAG}_literal.json 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_literal.json
