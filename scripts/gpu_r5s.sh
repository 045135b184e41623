# Round 5: excluded-dish clamp in the register draw -- z-pass timing on
# configs[3] and configs[1], then the full GPU suite.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5s}
for c in c4 c2; do
  ZP_CONFIG=$c timeout -k 10 180 python -u scripts/zprobe.py > gpurun_out/${TAG}_zprobe_$c.json 2>&1 || { tail -5 gpurun_out/${TAG}_zprobe_$c.json; exit 1; }
  tail -1 gpurun_out/${TAG}_zprobe_$c.json
done
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
