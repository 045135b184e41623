# Round 4: the run kernel's phase timers (MVC_RUN_PROF build) at the literal
# (warm, dense movers) and at configs[1]'s cold sweep 0.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
MVC_HIP_LIB=build_variants/runprof/libmvc_hip.so timeout -k 10 300 python scripts/r3_probe.py shapes > gpurun_out/r4t_runprof.log 2>&1
echo "rc=$?"; grep -E "runprof|tag" gpurun_out/r4t_runprof.log | cut -c1-260
