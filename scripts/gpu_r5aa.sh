# Round 5: the register draw's per-view scalars loaded one view ahead --
# z-path / phase-A parity, then z-pass timing at configs[3] (two runs).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5aa}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "zpath or phase_a or golden or config4" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  ZP_REPS=20 timeout -k 10 180 python -u scripts/zprobe.py > gpurun_out/${TAG}_zprobe_$r.json 2>&1 || { tail -5 gpurun_out/${TAG}_zprobe_$r.json; exit 1; }
  tail -1 gpurun_out/${TAG}_zprobe_$r.json
done
