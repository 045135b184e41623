# Round 5: producer without the matrix pipe (timing ablation); kernel trace
# of the reference's own call (N = 200, parallel schedule).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5m}
for v in nomfma nomfma_nostore; do
  export MVC_HIP_LIB=$PWD/build_variants/$v/libmvc_hip.so
  timeout -k 10 200 python -u scripts/zprobe.py >> gpurun_out/${TAG}_zprobe.log 2>&1 || { echo "zprobe $v failed"; exit 1; }
done
unset MVC_HIP_LIB
cat gpurun_out/${TAG}_zprobe.log
timeout -k 10 120 python -u scripts/newsim_prof.py > gpurun_out/${TAG}_newsim.log 2>&1 || exit 1
cat gpurun_out/${TAG}_newsim.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_nsprof -o run --output-format csv -- \
  python3 scripts/newsim_prof.py > gpurun_out/${TAG}_nsprof.log 2>&1 || { echo "ns prof failed"; exit 1; }
grep newsim gpurun_out/${TAG}_nsprof.log
find gpurun_out/${TAG}_nsprof -name "*kernel_trace.csv" -delete
