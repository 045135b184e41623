# Round 4: exact kernel v3 (LDS-only step barriers, y prefetch, batched MH sums):
# parity, the probe; the Reuters fin-kernel phase profile (MVC_RUN_PROF build).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "exact or dropin or c_abi" \
  > gpurun_out/r4m_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r4m_pytest.log; [ $rc -eq 0 ] || exit 1
for C in 1024 2048 4096; do timeout -k 10 200 python scripts/exact_probe.py $C >> gpurun_out/r4m_exact.json 2>> gpurun_out/r4m_exact.log || exit 1; done &&
MVC_EXACT_PROF=1 timeout -k 10 200 python scripts/exact_probe.py 2048 >> gpurun_out/r4m_exact.json 2>> gpurun_out/r4m_exact.log &&
cat gpurun_out/r4m_exact.json gpurun_out/r4m_exact.log &&
MVC_HIP_LIB=build_variants/runprof/libmvc_hip.so timeout -k 10 300 python scripts/reuters_run.py --sweeps 2 --chains 1 --ari-every 100 \
  --budget-s 200 --resume scratch/reuters_state.npz > gpurun_out/r4m_wideprof.log 2>&1; tail -8 gpurun_out/r4m_wideprof.log
