# Round 5: the register draw reduces the first mover itself (no mvc_seq_first_kernel launch) --
# full GPU suite, the reference call, configs[1] cold, the literal.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5av}
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
timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2>&1 || exit 1
grep -o '"value": [0-9.]*, "unit": "sweeps/s", "n_gpus": 1, "steps": 50, "warmup": 5, "ms_per_step": [0-9.]*' gpurun_out/${TAG}_bench.json
