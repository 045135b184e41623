# Round 5 measurement at HEAD: the bench line with every extra leg, the
# rocprofv3 kernel summary of the headline run, and the z-pass PMC.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5r}
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench_legs.log || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench_legs.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print(d['value'],d['roofline'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_prof_bench.json 2>&1 || { echo "rocprof failed"; exit 1; }
find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" -delete
bash scripts/gpu_pmc_z.sh ${TAG} || exit 1
echo done
