# Round 4: where a Reuters sweep's time goes (one chain, two sweeps from the
# r4i state, rocprofv3 kernel summary), then the 8-chain trajectory continued.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4k_prof -o run --output-format csv -- \
  python3 scripts/reuters_run.py --sweeps 2 --chains 1 --ari-every 100 --budget-s 200 --resume scratch/reuters_state.npz \
  > gpurun_out/r4k_prof.log 2>&1 &&
tail -3 gpurun_out/r4k_prof.log &&
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r4k_prof/**/*kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(r["Name"][:60], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6, 1), "ms", round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
find gpurun_out/r4k_prof -name "*kernel_trace.csv" -delete
timeout -k 10 1000 python scripts/reuters_run.py --sweeps 2000 --chains 8 --budget-s 840 --ari-every 10 \
  --resume scratch/reuters_state.npz --save gpurun_out/r4k_reuters_state.npz > gpurun_out/r4k_reuters.log 2>&1
echo "reuters rc=$?"; tail -2 gpurun_out/r4k_reuters.log | cut -c1-250
