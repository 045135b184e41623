cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_reu -o run --output-format csv -- python3 -u scripts/reuters_run.py --sweeps 2 --chains 1 --ari-every 5 --budget-s 60 > gpurun_out/reu_prof.log 2>&1 || { tail gpurun_out/reu_prof.log; exit 1; }
cat gpurun_out/reu_prof.log | grep sweep
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof_reu/**/run_kernel_stats.csv', recursive=True) or glob.glob('gpurun_out/prof_reu/*kernel_stats.csv')
rows = list(csv.DictReader(open(f[0])))
for r in rows[:12]:
    print(r['Name'][:50].ljust(50), r['Calls'], round(float(r['TotalDurationNs'])/1e6, 1), 'ms', round(float(r['AverageNs'])/1e3, 1), 'us')
PY
