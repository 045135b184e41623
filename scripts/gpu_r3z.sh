#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/newsim_probe.py > gpurun_out/newsim_r3z.json 2> gpurun_out/newsim_r3z.err \
    || { echo "probe failed"; tail gpurun_out/newsim_r3z.err; exit 1; }
cat gpurun_out/newsim_r3z.json
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3z -o run --output-format csv -- \
    python3 -c "
import sys; sys.path.insert(0,'multiview-clustering_amd')
import mvc_amd
from mvc_amd import data
y,_=data.new_simulation(1999)
for C in (1, 2048):
    s=mvc_amd.Sampler(y, seed=1999, mode='exact', n_chains=C); s.sweep(100); s.synchronize(); s.close()
" > gpurun_out/prof_r3z.log 2>&1 || { echo "rocprof failed"; exit 1; }
grep -i "exact" gpurun_out/prof_r3z/run_kernel_trace.csv | python3 -c "
import sys,csv
rows=list(csv.reader(sys.stdin))
d=[(int(r[-2])-int(r[-3])) if r[-2].isdigit() else 0 for r in rows]
" 2>/dev/null; head -5 gpurun_out/prof_r3z/run_kernel_stats.csv
echo done
