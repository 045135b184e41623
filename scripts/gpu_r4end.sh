# Round 4 end (HEAD after the value-prediction change): the full GPU suite (as the driver runs it), smoke, the driver's
# bench command and its rocprofv3 kernel summary; then the exact kernel's LDS
# PMC pass and the run kernel's phase timers.  Each step under its own limit.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs > gpurun_out/r4end_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r4end_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4end_smoke.log 2>&1 && tail -1 gpurun_out/r4end_smoke.log &&
timeout -k 10 600 python bench.py > gpurun_out/r4end_bench.json 2> gpurun_out/r4end_bench.log &&
echo "bench ok" && tail -c 300 gpurun_out/r4end_bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4end_prof -o r4end -- python3 bench.py --no-extras --no-cpu-baseline --steps 20 > gpurun_out/r4end_prof_bench.json 2> gpurun_out/r4end_prof.log &&
find gpurun_out/r4end_prof -name "*kernel_trace.csv" -delete && echo "prof ok" || exit 1
for C in 2048 4096; do timeout -k 10 200 python scripts/exact_probe.py $C >> gpurun_out/r4end_exact.json 2>> gpurun_out/r4end_exact.log || exit 1; done
cat gpurun_out/r4end_exact.json
MVC_HIP_LIB=build_variants/runprof/libmvc_hip.so timeout -k 10 300 python scripts/r3_probe.py shapes > gpurun_out/r4end_runprof.log 2>&1
echo "runprof rc=$?"; grep -E "runprof|tag" gpurun_out/r4end_runprof.log | cut -c1-260
GPU_MAX_HW_QUEUES=32 timeout -k 10 300 python bench.py --leg newsim_chains > gpurun_out/r4end_q32.json 2> gpurun_out/r4end_q32.log && cat gpurun_out/r4end_q32.json | cut -c1-600
