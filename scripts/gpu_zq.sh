# z-pass check: the producer / phase-A parity tests, then the headline bench
# (no extra legs) under rocprofv3 --kernel-trace --stats.
# usage: gpu_zq.sh TAG ["<pytest -k expr>"]
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=$1; KEXPR=${2:-"zpath or phase_a or config4 or lpall"}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs -k "$KEXPR" \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_bench.json 2>gpurun_out/${TAG}_bench.err || { echo "rocprof failed"; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" -delete
python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().split('\n')[-1]);print(d['value'],d['ms_per_step'],d['roofline'])"
find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" -exec head -8 {} \;
