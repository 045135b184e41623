# Round 4: the fin kernel's LDS-resident evaluation and leaf-reusing birth draws:
# the repair parity tests, the Reuters corpus test, the fin phase profile,
# then the 8-chain Reuters sweeps from the saved state.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_reuters.py -x -v --timeout 600 --timeout-method thread \
  -k "global_wide or repair or chains or reuters or config3 or parallel_golden or capacity" > gpurun_out/r4o_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r4o_pytest.log; [ $rc -eq 0 ] || exit 1
MVC_HIP_LIB=build_variants/runprof/libmvc_hip.so timeout -k 10 300 python scripts/reuters_run.py --sweeps 2 --chains 1 --ari-every 100 \
  --budget-s 200 --resume scratch/reuters_state.npz > gpurun_out/r4o_wideprof.log 2>&1; grep -E "wideprof|sweep" gpurun_out/r4o_wideprof.log | cut -c1-250
timeout -k 10 400 python scripts/reuters_run.py --sweeps 20 --chains 8 --ari-every 10 --budget-s 240 \
  --resume scratch/reuters_state.npz > gpurun_out/r4o_reuters.log 2>&1; echo "rc=$?"; tail -3 gpurun_out/r4o_reuters.log | cut -c1-250
