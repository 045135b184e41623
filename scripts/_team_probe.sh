cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "repair or chains or config2 or golden or live_oracle or warm or dish_block" > gpurun_out/pt_team.log 2>&1 || { tail -30 gpurun_out/pt_team.log; exit 1; }
tail -3 gpurun_out/pt_team.log
for T in 1 2 4; do
  echo "== team $T"
  MVC_TEAM=$T timeout -k 10 120 python -u scripts/coldstart.py --config c2 --sweeps 3 || exit 1
  MVC_TEAM=$T timeout -k 10 120 python -u scripts/coldstart.py --config ns --warm --sweeps 2 --budget-s 30 || exit 1
  MVC_TEAM=$T timeout -k 10 120 python -u scripts/coldstart.py --config c4s --sweeps 2 --budget-s 40 || exit 1
done
