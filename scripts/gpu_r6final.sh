# Round 6: the full GPU suite and smoke (round-end shape), then optionally
# scripts/gpu_r5r.sh (bench line with every leg + rocprof + z-pass PMC).
# usage: gpu_r6final.sh TAG [bench]
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r6final}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
if [ "$2" = "bench" ]; then bash scripts/gpu_r5r.sh ${TAG} || exit 1; fi
