# Round 5: full GPU suite at HEAD, then phase-A timing and the bench line.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5j}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u scripts/zprobe.py > gpurun_out/${TAG}_zprobe.log 2>&1 || exit 1
cat gpurun_out/${TAG}_zprobe.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extras > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print(d['value'],d['roofline'],d['kernel_ms_per_sweep'])"
