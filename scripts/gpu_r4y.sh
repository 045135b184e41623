# Round 4: a live GPU context in the parent vs the bench's child legs.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python scripts/parent_ctx_probe.py > gpurun_out/r4y.json 2> gpurun_out/r4y.log || exit 1
timeout -k 10 300 python scripts/parent_ctx_probe.py reset >> gpurun_out/r4y.json 2>> gpurun_out/r4y.log || exit 1
cat gpurun_out/r4y.json | cut -c1-600
