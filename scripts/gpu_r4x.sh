# Round 4: why the bench's New_Simulation chains leg ran at half the speed it
# shows alone: the leg alone, after the configs[4] leg (164 GB, MFMA-heavy),
# and the exact probe over the bench's sweep range.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python scripts/exact_probe.py 2048 200 250 500 > gpurun_out/r4x.json 2> gpurun_out/r4x.log || exit 1
timeout -k 10 300 python bench.py --leg newsim_chains >> gpurun_out/r4x.json 2>> gpurun_out/r4x.log || exit 1
timeout -k 10 300 python bench.py --leg configs4_full_gpu >> gpurun_out/r4x.json 2>> gpurun_out/r4x.log || exit 1
timeout -k 10 300 python bench.py --leg newsim_chains >> gpurun_out/r4x.json 2>> gpurun_out/r4x.log || exit 1
cat gpurun_out/r4x.json | cut -c1-700
