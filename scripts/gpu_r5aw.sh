# Round 5: the first batch of repair rounds of a small chain (MVC_SMALL_ROUNDS)
# at the reference's call.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5aw}
for r in 4 2 3 6 4; do
  MVC_SMALL_ROUNDS=$r timeout -k 10 300 python3 bench.py --leg newsim_call > gpurun_out/${TAG}_ns_r$r.json 2>&1 || exit 1
  echo "rounds $r: $(tail -1 gpurun_out/${TAG}_ns_r$r.json | cut -c90-190)"
done
