# configs[4] producer check: the dish-block tests, then the configs4 leg with
# the XCD-grouped dish-block launch and with one launch per block
# (MVC_PATH big_group=0), then the grouped leg under rocprofv3 --stats.
# usage: gpu_c4.sh TAG
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=$1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -rs \
  -k "dish_block or config5" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py --leg configs4_full_gpu > gpurun_out/${TAG}_c4_group.json 2> gpurun_out/${TAG}_c4_group.err || { tail -5 gpurun_out/${TAG}_c4_group.err; exit 1; }
cat gpurun_out/${TAG}_c4_group.json
MVC_PATH=big_group=0 timeout -k 10 400 python -u bench.py --leg configs4_full_gpu > gpurun_out/${TAG}_c4_sep.json 2> gpurun_out/${TAG}_c4_sep.err || { tail -5 gpurun_out/${TAG}_c4_sep.err; exit 1; }
cat gpurun_out/${TAG}_c4_sep.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c4prof -o run --output-format csv -- \
    python3 bench.py --leg configs4_full_gpu > gpurun_out/${TAG}_c4_prof.json 2>&1 || { echo "rocprof failed"; exit 1; }
find gpurun_out/${TAG}_c4prof -name "*kernel_trace.csv" -delete
find gpurun_out/${TAG}_c4prof -name "*kernel_stats.csv" -exec head -12 {} \;
