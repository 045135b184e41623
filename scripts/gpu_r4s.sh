# Round 4: the exact kernel's table-capacity shrink (build_variants/shr:
# MVC_EXACT_SHRINK=1): parity through the shrink, then the probe (default,
# shrink, shrink + 3 waves per SIMD) at 2,048 / 4,096 chains.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
MVC_HIP_LIB=build_variants/shr/libmvc_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 \
  --timeout-method thread -k "exact or dropin or c_abi" > gpurun_out/r4s_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r4s_pytest.log; [ $rc -eq 0 ] || exit 1
for L in multiview-clustering_amd/lib build_variants/shr build_variants/ex3s; do
  for C in 2048 4096; do
    MVC_HIP_LIB=$L/libmvc_hip.so timeout -k 10 200 python scripts/exact_probe.py $C >> gpurun_out/r4s_exact.json 2>> gpurun_out/r4s_exact.log || exit 1
  done
done
cat gpurun_out/r4s_exact.json
