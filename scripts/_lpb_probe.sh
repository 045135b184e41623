cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "lpall_batches or zpath2 or config4 or repair_team" > gpurun_out/pt_lpb.log 2>&1 || { tail -30 gpurun_out/pt_lpb.log; exit 1; }
tail -2 gpurun_out/pt_lpb.log
for B in 0 262144 131072 65536 32768 16384; do
  echo "== batch $B"
  MVC_LPB_BATCH=$B timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d.get('phase_ms', d.get('timers')))" || exit 1
done
