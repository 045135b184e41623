# Round 5: producer waves per CU / ring depth variants (phase-A timing),
# plus phase-A parity of each variant.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5c}
for v in default w8rp16 w4rp16 w4rp8; do
  if [ $v = default ]; then unset MVC_HIP_LIB; else export MVC_HIP_LIB=$PWD/build_variants/$v/libmvc_hip.so; fi
  timeout -k 10 200 python -u scripts/zprobe.py >> gpurun_out/${TAG}_zprobe.log 2>&1 || { echo "zprobe $v failed"; exit 1; }
done
cat gpurun_out/${TAG}_zprobe.log
for v in w8rp16 w4rp16 w4rp8; do
  export MVC_HIP_LIB=$PWD/build_variants/$v/libmvc_hip.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "zpath2 or phase_a or config4" > gpurun_out/${TAG}_pytest_$v.log 2>&1 || { echo "parity $v failed"; tail -5 gpurun_out/${TAG}_pytest_$v.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pytest_$v.log
done
