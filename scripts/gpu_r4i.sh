# Round 4: repair timings (the literal warm sweeps and configs[1] cold, with
# and without value prediction), the run kernel's PMC passes, then the Reuters
# 8-chain trajectory on the grid-wide evaluation (state saved for a resume).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python scripts/r3_probe.py shapes > gpurun_out/r4i_shapes.log 2>&1 &&
timeout -k 10 300 env MVC_VP=0 python scripts/r3_probe.py shapes > gpurun_out/r4i_shapes_vp0.log 2>&1 &&
echo "shapes ok" && cat gpurun_out/r4i_shapes.log gpurun_out/r4i_shapes_vp0.log &&
bash scripts/gpu_pmc_run.sh r4i > gpurun_out/r4i_pmc_summary.json 2> gpurun_out/r4i_pmc.err &&
echo "pmc ok" &&
timeout -k 10 720 python scripts/reuters_run.py --sweeps 2000 --chains 8 --budget-s 600 --ari-every 10 \
    --save gpurun_out/r4i_reuters_state.npz > gpurun_out/r4i_reuters.log 2>&1 ;
echo "reuters rc=$?"; tail -3 gpurun_out/r4i_reuters.log
