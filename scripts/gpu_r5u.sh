# Round 5: kernel summary of the reference's own call (N = 200, parallel
# schedule, one chain) at HEAD, after the births moved into the run kernel.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5u}
timeout -k 10 120 python -u scripts/newsim_prof.py > gpurun_out/${TAG}_newsim.log 2>&1 || exit 1
cat gpurun_out/${TAG}_newsim.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_nsprof -o run --output-format csv -- \
  python3 scripts/newsim_prof.py > gpurun_out/${TAG}_nsprof.log 2>&1 || { echo "ns prof failed"; exit 1; }
grep newsim gpurun_out/${TAG}_nsprof.log
TAG=$TAG python3 - <<'PY'
import csv, glob, collections, os
f = [p for p in glob.glob("gpurun_out/%s_nsprof/**/*kernel_trace.csv" % os.environ["TAG"], recursive=True)][0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the timed call's last 200 sweeps: kernel sequence and gaps between launches
names = [r["Kernel_Name"][:40] for r in rows]
print("kernels:", len(rows))
tail = rows[-3000:]
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tail)
span = int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])
print("tail 3000 launches: busy %.3f ms of %.3f ms" % (busy / 1e6, span / 1e6))
seq = collections.Counter(r["Kernel_Name"][:40] for r in tail)
print(seq.most_common(12))
for r in rows[-40:]:
    print(r["Kernel_Name"][:40], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), int(r["Start_Timestamp"]) % 10**9)
PY
find gpurun_out/${TAG}_nsprof -name "*kernel_trace.csv" -delete
