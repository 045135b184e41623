# Round 4: the exact schedule on the New_Simulation shape: timing, then its
# sweep kernel's PMC passes.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 python scripts/exact_probe.py 2048 > gpurun_out/r4j_exact.json 2> gpurun_out/r4j_exact.log &&
MVC_EXACT_PROF=1 timeout -k 10 200 python scripts/exact_probe.py 2048 >> gpurun_out/r4j_exact.json 2>> gpurun_out/r4j_exact.log &&
timeout -k 10 200 python scripts/exact_probe.py 1024 >> gpurun_out/r4j_exact.json 2>> gpurun_out/r4j_exact.log &&
cat gpurun_out/r4j_exact.json gpurun_out/r4j_exact.log &&
bash scripts/gpu_pmc_exact.sh r4j > gpurun_out/r4j_pmc_exact.json 2> gpurun_out/r4j_pmc_exact.err &&
cat gpurun_out/r4j_pmc_exact.json
