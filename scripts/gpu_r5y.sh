# Round 5: the dish-block producer's A-fragments as 16-byte loads (two
# k-steps per load, lane swaps): parity cases, then the configs[4] leg with
# 8 and 16 pair loads in flight (build_variants/rp16), kernel summary.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5y}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_synthetic.py -x -v --timeout 300 --timeout-method thread \
  -k "dish_block or config4 or configs4" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --leg configs4_full_gpu > gpurun_out/${TAG}_c5.json 2>&1 || exit 1
echo "rp8: $(tail -1 gpurun_out/${TAG}_c5.json | cut -c200-420)"
MVC_HIP_LIB=$PWD/build_variants/rp16/libmvc_hip.so timeout -k 10 300 python3 bench.py --leg configs4_full_gpu > gpurun_out/${TAG}_c5_rp16.json 2>&1 || exit 1
echo "rp16: $(tail -1 gpurun_out/${TAG}_c5_rp16.json | cut -c200-420)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c5prof -o run --output-format csv -- \
  python3 bench.py --leg configs4_full_gpu > gpurun_out/${TAG}_c5prof.log 2>&1 || { echo "prof failed"; exit 1; }
find gpurun_out/${TAG}_c5prof -name "*kernel_trace.csv" -delete
