# Round 5: configs[4] draw alternatives (row draw with per-lane view scalars;
# the checkpoint draw with its score scratch) and the row draw at configs[3].
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5h}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "zpath2 or config5_shape" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --leg configs4_full_gpu > gpurun_out/${TAG}_c5leg.json 2>&1 || { echo "c5 leg failed"; exit 1; }
tail -1 gpurun_out/${TAG}_c5leg.json | cut -c1-300
MVC_ZDRAW_LDS=1 MVC_ZSC_MAX_MB=8192 timeout -k 10 300 python3 bench.py --leg configs4_full_gpu > gpurun_out/${TAG}_c5leg_sc.json 2>&1 || { echo "c5 leg sc failed"; exit 1; }
tail -1 gpurun_out/${TAG}_c5leg_sc.json | cut -c1-300
MVC_ZDRAW_ROW=1 timeout -k 10 200 python -u scripts/zprobe.py >> gpurun_out/${TAG}_zprobe.log 2>&1 || exit 1
cat gpurun_out/${TAG}_zprobe.log
