# Round 5: the MH kernel phase marks (MVC_HYP_PROF build): configs[3] warm and the reference call shape.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5ac}
MVC_HIP_LIB=$PWD/build_variants/hypprof/libmvc_hip.so timeout -k 10 200 python -u scripts/hyp_prof.py > gpurun_out/${TAG}_hypprof.log 2>&1 || { tail -5 gpurun_out/${TAG}_hypprof.log; exit 1; }
cat gpurun_out/${TAG}_hypprof.log
HP_CONFIG=ns200 MVC_HIP_LIB=$PWD/build_variants/hypprof/libmvc_hip.so timeout -k 10 200 python -u scripts/hyp_prof.py > gpurun_out/${TAG}_hypprof_ns.log 2>&1 || { tail -5 gpurun_out/${TAG}_hypprof_ns.log; exit 1; }
cat gpurun_out/${TAG}_hypprof_ns.log
