# Round 4 end: the run kernel's PMC passes after the value-prediction change.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash scripts/gpu_pmc_run.sh r4pmc > gpurun_out/r4pmc_summary.json 2> gpurun_out/r4pmc.err; rc=$?
rm -rf gpurun_out/pmcr_r4pmc_*/
cat gpurun_out/r4pmc_summary.json; exit $rc
