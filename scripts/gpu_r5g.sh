# Round 5: row draw (VGPR exp coefficients, two waves per SIMD in its LDS
# form): parity, configs[4] leg; and the row draw forced at configs[3] (T = 64)
# against the register draw (phase-A timing).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5g}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "zpath2 or config5_shape" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --leg configs4_full_gpu > gpurun_out/${TAG}_c5leg.json 2>&1 || { echo "c5 leg failed"; exit 1; }
tail -1 gpurun_out/${TAG}_c5leg.json | cut -c1-400
timeout -k 10 200 python -u scripts/zprobe.py >> gpurun_out/${TAG}_zprobe.log 2>&1 || exit 1
MVC_ZDRAW_ROW=1 timeout -k 10 200 python -u scripts/zprobe.py >> gpurun_out/${TAG}_zprobe.log 2>&1 || exit 1
MVC_ZDRAW_ROW=1 MVC_ZROW_LDS=0 timeout -k 10 200 python -u scripts/zprobe.py >> gpurun_out/${TAG}_zprobe.log 2>&1 || exit 1
cat gpurun_out/${TAG}_zprobe.log
