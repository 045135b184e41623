# Round 5: non-temporal cache hints on the producer's y loads / lp stores
# (build_variants ynt, stnt, both) -- z-pass timing at configs[3].
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5ab}
for v in default ynt stnt both default; do
  if [ $v = default ]; then unset MVC_HIP_LIB; else export MVC_HIP_LIB=$PWD/build_variants/$v/libmvc_hip.so; fi
  ZP_REPS=20 timeout -k 10 180 python -u scripts/zprobe.py >> gpurun_out/${TAG}_zprobe.log 2>&1 || { echo "zprobe $v failed"; tail -3 gpurun_out/${TAG}_zprobe.log; exit 1; }
done
cat gpurun_out/${TAG}_zprobe.log
