#!/bin/bash
# the New_Simulation.R call: wall time in both schedules, then its kernels under rocprofv3
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 120 python3 -u scripts/r3_probe.py newsim 2000 > gpurun_out/r3m_newsim.log 2>&1 || { echo "newsim failed"; tail gpurun_out/r3m_newsim.log; exit 1; }
cat gpurun_out/r3m_newsim.log
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3m -o run --output-format csv -- \
    python3 scripts/r3_probe.py newsim 2000 > gpurun_out/prof_r3m.log 2>&1 || { echo "rocprof failed"; exit 1; }
head -30 gpurun_out/prof_r3m/run_kernel_stats.csv | cut -c1-160
timeout -k 10 420 python3 -u scripts/coldstart.py --config c4 --sweeps 40 --budget-s 330 > gpurun_out/r3m_cold_c4.log 2>&1
rc=$?; echo "coldstart exit $rc"; tail -4 gpurun_out/r3m_cold_c4.log
