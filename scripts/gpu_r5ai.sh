# Round 5: MH kernel with the view offsets, hyperparameters and first-dish values staged --
# full GPU suite, headline bench (no extras) and its kernel summary.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5ai}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2>&1 || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_prof_bench.json 2>&1 || { echo "rocprof failed"; exit 1; }
find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" -delete
timeout -k 10 120 python -u scripts/newsim_prof.py > gpurun_out/${TAG}_newsim.log 2>&1 || exit 1
head -1 gpurun_out/${TAG}_newsim.log
