# Round 5: the run kernel's LDS layout with room to double T (MVC_RUN_GROW):
# the literal with 1, 16 and 64 chains (chain-batched repair), and configs[1]'s
# cold start, with and without it.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5t}
for g in 1 0; do
  MVC_RUN_GROW=$g timeout -k 10 200 python3 bench.py --leg north_star_literal_gpu > gpurun_out/${TAG}_lit1_grow$g.json 2>&1 || exit 1
  tail -1 gpurun_out/${TAG}_lit1_grow$g.json | cut -c1-300
  MVC_RUN_GROW=$g timeout -k 10 300 python -u scripts/ns_chains.py 16 64 > gpurun_out/${TAG}_chains_grow$g.log 2>&1 || { tail -3 gpurun_out/${TAG}_chains_grow$g.log; exit 1; }
  cat gpurun_out/${TAG}_chains_grow$g.log
  MVC_RUN_GROW=$g timeout -k 10 200 python3 bench.py --leg cold_start_gpu > gpurun_out/${TAG}_cold_grow$g.json 2>&1 || exit 1
  tail -1 gpurun_out/${TAG}_cold_grow$g.json | cut -c1-400
done
