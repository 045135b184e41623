# Round 4: does the exact kernel gain from 3 / 4 waves per SIMD (register
# budget 168 / 128)?  4,096 chains at n = 100 (LDS allows > 8 chains per CU)
# and n = 200, against the default build.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for L in multiview-clustering_amd/lib build_variants/ex3 build_variants/ex4; do
  for N in 100 200; do
    MVC_HIP_LIB=$L/libmvc_hip.so timeout -k 10 200 python scripts/exact_probe.py 4096 $N >> gpurun_out/r4r_exact.json 2>> gpurun_out/r4r_exact.log || exit 1
  done
done
cat gpurun_out/r4r_exact.json
MVC_HIP_LIB=build_variants/runprof/libmvc_hip.so timeout -k 10 300 python scripts/reuters_run.py --sweeps 1 --chains 1 --ari-every 100 \
  --budget-s 200 --resume scratch/reuters_state.npz > gpurun_out/r4r_wideprof.log 2>&1; grep -E "wideprof|sweep" gpurun_out/r4r_wideprof.log | cut -c1-250
