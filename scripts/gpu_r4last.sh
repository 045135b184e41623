# Round 4 last check: the full GPU suite and smoke at HEAD.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs > gpurun_out/r4last_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r4last_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4last_smoke.log 2>&1 && tail -1 gpurun_out/r4last_smoke.log
