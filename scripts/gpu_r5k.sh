# Round 5: all-views producer epilogue bisection (timing-only ablations).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5k}
for v in default nomax noend nostore nsnm noepi; do
  if [ $v = default ]; then unset MVC_HIP_LIB; else export MVC_HIP_LIB=$PWD/build_variants/$v/libmvc_hip.so; fi
  timeout -k 10 200 python -u scripts/zprobe.py >> gpurun_out/${TAG}_zprobe.log 2>&1 || { echo "zprobe $v failed"; exit 1; }
done
cat gpurun_out/${TAG}_zprobe.log
