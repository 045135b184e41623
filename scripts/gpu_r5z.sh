# Round 5: the row draw's per-view scalars loaded once per round -- the
# z-path parity cases, configs[4] at full size (test), its bench leg and
# kernel summary.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5z}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_synthetic.py -x -v --timeout 300 --timeout-method thread \
  -k "zpath or row or config5 or dish_block or phase_a" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --leg configs4_full_gpu > gpurun_out/${TAG}_c5.json 2>&1 || exit 1
echo "$(tail -1 gpurun_out/${TAG}_c5.json | cut -c200-420)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c5prof -o run --output-format csv -- \
  python3 bench.py --leg configs4_full_gpu > gpurun_out/${TAG}_c5prof.log 2>&1 || { echo "prof failed"; exit 1; }
find gpurun_out/${TAG}_c5prof -name "*kernel_trace.csv" -delete
