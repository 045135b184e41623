# Round 5: G-form producer + register draw -- parity of the phase-A paths,
# then phase-A timing: G form (2 and 3 waves per SIMD draws) vs lp form.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5s}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "zpath2 or phase_a or config4 or mfma or warm_start or parallel_golden or generic or capacity" \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u scripts/zprobe.py >> gpurun_out/${TAG}_zprobe.log 2>&1 || exit 1
MVC_GFORM=0 timeout -k 10 200 python -u scripts/zprobe.py >> gpurun_out/${TAG}_zprobe.log 2>&1 || exit 1
MVC_HIP_LIB=$PWD/build_variants/gminb3/libmvc_hip.so timeout -k 10 200 python -u scripts/zprobe.py >> gpurun_out/${TAG}_zprobe.log 2>&1 || exit 1
cat gpurun_out/${TAG}_zprobe.log
