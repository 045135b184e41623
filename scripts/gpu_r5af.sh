# Round 5: value prediction and the stay limit at three shapes -- the
# reference's call (N = 200), configs[1] cold (N = 100k) and the literal.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5af}
k=0
for cfg in "MVC_X=0" "MVC_VP=0" "MVC_VP=0 MVC_RUN_LIMIT=2" "MVC_VP=0 MVC_RUN_LIMIT=4" "MVC_VP=0 MVC_RUN_LIMIT=8" "MVC_VP=0 MVC_RUN_LIMIT=16" "MVC_RUN_LIMIT=8"; do
  k=$((k+1))
  env $cfg NS_SWEEPS=2000 timeout -k 10 120 python -u scripts/newsim_prof.py > gpurun_out/${TAG}_ns$k.log 2>&1 || { echo "$cfg failed"; tail -3 gpurun_out/${TAG}_ns$k.log; exit 1; }
  echo "newsim $cfg: $(grep 'newsim parallel' gpurun_out/${TAG}_ns$k.log)"
done
for cfg in "MVC_X=0" "MVC_VP=0"; do
  k=$((k+1))
  env $cfg timeout -k 10 200 python3 bench.py --leg cold_start_gpu > gpurun_out/${TAG}_cold$k.json 2>&1 || exit 1
  echo "cold $cfg: $(tail -1 gpurun_out/${TAG}_cold$k.json | cut -c100-330)"
  env $cfg timeout -k 10 200 python3 bench.py --leg north_star_literal_gpu > gpurun_out/${TAG}_lit$k.json 2>&1 || exit 1
  echo "literal $cfg: $(tail -1 gpurun_out/${TAG}_lit$k.json | cut -c80-200)"
done
