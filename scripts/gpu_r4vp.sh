# Round 4: value prediction with the overlay's dish lookups in registers:
# the repair / vp parity tests, the literal and configs[1] timings, the phase timers.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "value_prediction or repair or chains or parallel_golden or stats_bitwise or warm" > gpurun_out/r4vp_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4vp_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/r3_probe.py shapes > gpurun_out/r4vp_shapes.log 2>&1 && cut -c1-200 gpurun_out/r4vp_shapes.log
MVC_HIP_LIB=build_variants/runprof/libmvc_hip.so timeout -k 10 300 python scripts/r3_probe.py shapes > gpurun_out/r4vp_runprof.log 2>&1
grep -E "runprof moves|tag" gpurun_out/r4vp_runprof.log | cut -c1-230
