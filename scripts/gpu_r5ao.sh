# Round 5: configs[1] cold start (N = 100k) under the repair's switches.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5ao}
k=0
for cfg in "MVC_X=0" "MVC_SMALL_N_PLAIN=200000" "MVC_RUN_LIMIT=16" "MVC_RUN_LIMIT=256" "MVC_VP=0 MVC_RUN_LIMIT=16" "MVC_RUN_WAVES=8"; do
  k=$((k+1))
  env $cfg timeout -k 10 200 python3 bench.py --leg cold_start_gpu > gpurun_out/${TAG}_cold$k.json 2>&1 || { echo "$cfg failed"; tail -3 gpurun_out/${TAG}_cold$k.json; exit 1; }
  echo "cold $cfg: $(tail -1 gpurun_out/${TAG}_cold$k.json | cut -c100-300)"
done
