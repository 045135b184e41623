# Round 5: branch-free lane-parallel log-gammas in the MH kernel's EPPF --
# full GPU suite, MH phase marks (profiling build), headline bench, the
# reference's call, kernel summary.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5ak}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
HP_CONFIG=ns200 MVC_HIP_LIB=$PWD/build_variants/hypprof/libmvc_hip.so timeout -k 10 200 python -u scripts/hyp_prof.py > gpurun_out/${TAG}_hypprof_ns.log 2>&1 || { tail -5 gpurun_out/${TAG}_hypprof_ns.log; exit 1; }
cat gpurun_out/${TAG}_hypprof_ns.log
timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2>&1 || exit 1
grep -o '"value": [0-9.]*, "unit": "sweeps/s", "n_gpus": 1, "steps": 50, "warmup": 5, "ms_per_step": [0-9.]*' gpurun_out/${TAG}_bench.json
timeout -k 10 120 python -u scripts/newsim_prof.py > gpurun_out/${TAG}_newsim.log 2>&1 || exit 1
head -1 gpurun_out/${TAG}_newsim.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_prof_bench.json 2>&1 || { echo "rocprof failed"; exit 1; }
find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" -delete
