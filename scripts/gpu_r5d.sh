# Round 5: the row draw (16 lanes per customer, T > 64): parity on every
# z-path shape, the configs[4]-shaped reduced test, then the configs[4] leg.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5d}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "zpath2 or config5_shape or dish_block or capacity_growth or phase_a" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_synthetic.py -x -v --timeout 500 --timeout-method thread \
  > gpurun_out/${TAG}_pytest_synth.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest_synth.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c5prof -o run --output-format csv -- \
  python3 bench.py --leg configs4_full_gpu > gpurun_out/${TAG}_c5prof.log 2>&1 || { echo "c5 prof failed"; exit 1; }
tail -1 gpurun_out/${TAG}_c5prof.log | cut -c1-400
find gpurun_out/${TAG}_c5prof -name "*kernel_trace.csv" -delete
timeout -k 10 300 python3 bench.py --leg configs4_full_gpu > gpurun_out/${TAG}_c5leg.json 2>&1 || { echo "c5 leg failed"; exit 1; }
tail -1 gpurun_out/${TAG}_c5leg.json | cut -c1-600
MVC_ZROW_LDS=0 timeout -k 10 300 python3 bench.py --leg configs4_full_gpu > gpurun_out/${TAG}_c5leg_global.json 2>&1 || { echo "c5 leg global failed"; exit 1; }
tail -1 gpurun_out/${TAG}_c5leg_global.json | cut -c1-400
