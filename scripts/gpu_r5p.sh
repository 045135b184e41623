# Round 5: chain-batched literal at 128 chains, with the per-kernel split.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5p}
timeout -k 10 300 python -u scripts/ns_chains.py 64 128 > gpurun_out/${TAG}_ns_chains.log 2>&1 || { tail -3 gpurun_out/${TAG}_ns_chains.log; exit 1; }
cat gpurun_out/${TAG}_ns_chains.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
  python3 scripts/ns_chains.py 64 > gpurun_out/${TAG}_prof.log 2>&1 || { echo "prof failed"; exit 1; }
find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" -delete
