# Round 4: the driver's bench command, its rocprofv3 kernel summary, and the
# New_Simulation-shape probe.  Each step under its own limit; stop at the
# first failure.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python bench.py > gpurun_out/r4h_bench.json 2> gpurun_out/r4h_bench.log &&
echo "bench ok" && tail -c 600 gpurun_out/r4h_bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4h_prof -o r4h -- python3 bench.py --no-extras --no-cpu-baseline --steps 20 > gpurun_out/r4h_prof_bench.json 2> gpurun_out/r4h_prof.log &&
echo "prof ok" &&
timeout -k 10 300 python scripts/newsim_probe.py > gpurun_out/r4h_newsim.json 2> gpurun_out/r4h_newsim.log &&
echo "probe ok" && cat gpurun_out/r4h_newsim.json
