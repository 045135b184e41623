# Round 5: the run kernel's phase timers (MVC_RUN_PROF build) on the
# reference's call shape (N = 200, plain lane columns) and the literal.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5an}
MVC_HIP_LIB=$PWD/build_variants/runprof/libmvc_hip.so NS_SWEEPS=200 timeout -k 10 120 python -u scripts/newsim_prof.py > gpurun_out/${TAG}_runprof_ns.log 2>&1 || { tail -5 gpurun_out/${TAG}_runprof_ns.log; exit 1; }
grep runprof gpurun_out/${TAG}_runprof_ns.log | tail -6
