# Round 4: the New_Simulation chains leg with 32 vs 4 hardware queues.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
GPU_MAX_HW_QUEUES=32 timeout -k 10 300 python bench.py --leg newsim_chains > gpurun_out/r4z2.json 2> gpurun_out/r4z2.log || exit 1
GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python bench.py --leg newsim_chains >> gpurun_out/r4z2.json 2>> gpurun_out/r4z2.log || exit 1
cat gpurun_out/r4z2.json | cut -c1-600
