# Round 4 final: the full GPU suite (as the driver runs it), smoke, the
# driver's bench command and its rocprofv3 kernel summary.  Each step under
# its own limit; stop at the first failure.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs > gpurun_out/r4z_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r4z_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4z_smoke.log 2>&1 && tail -1 gpurun_out/r4z_smoke.log &&
timeout -k 10 900 python bench.py > gpurun_out/r4z_bench.json 2> gpurun_out/r4z_bench.log &&
echo "bench ok" && tail -c 400 gpurun_out/r4z_bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4z_prof -o r4z -- python3 bench.py --no-extras --no-cpu-baseline --steps 20 > gpurun_out/r4z_prof_bench.json 2> gpurun_out/r4z_prof.log &&
find gpurun_out/r4z_prof -name "*kernel_trace.csv" -delete && echo "prof ok"
