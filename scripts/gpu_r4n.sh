# Round 4: the Reuters 8-chain trajectory with the TOPICS columns zeroed
# (--drop-topics: a label-free score), from the cold start.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 1150 python scripts/reuters_run.py --sweeps 2000 --chains 8 --budget-s 1040 --ari-every 10 --drop-topics \
  --save gpurun_out/r4n_reuters_dt_state.npz > gpurun_out/r4n_reuters_dt.log 2>&1
echo "rc=$?"; tail -2 gpurun_out/r4n_reuters_dt.log | cut -c1-300
