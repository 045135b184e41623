# Round 5: the reference's call (N = 200, parallel schedule, one chain) under
# the repair's switches: value prediction off, lane columns off, no grid
# windows, run-kernel waves, stay limits; plus value-prediction step counts.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5ae}
k=0
for cfg in "MVC_X=0" "MVC_VP=0" "MVC_LC=0" "MVC_SMALL_N=256" "MVC_VP=0 MVC_SMALL_N=256" "MVC_RUN_WAVES=2" "MVC_RUN_LIMIT=4" "MVC_RUN_LIMIT=1024"; do
  k=$((k+1))
  env $cfg NS_SWEEPS=2000 timeout -k 10 120 python -u scripts/newsim_prof.py > gpurun_out/${TAG}_ns$k.log 2>&1 || { echo "$cfg failed"; tail -3 gpurun_out/${TAG}_ns$k.log; exit 1; }
  echo "$cfg: $(grep 'newsim parallel' gpurun_out/${TAG}_ns$k.log)"
done
MVC_VP_STATS=1 NS_SWEEPS=300 timeout -k 10 120 python -u scripts/newsim_prof.py > gpurun_out/${TAG}_vpstats.log 2>&1 || exit 1
grep "vp steps" gpurun_out/${TAG}_vpstats.log | tail -8
