cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_reuters.py -x -v --timeout 250 --timeout-method thread -k "capacity or reuters or chains or repair_shapes or config2" > gpurun_out/pt_ret.log 2>&1 || { tail -30 gpurun_out/pt_ret.log; exit 1; }
tail -2 gpurun_out/pt_ret.log
timeout -k 10 170 python -u scripts/reuters_run.py --sweeps 2 --chains 8 --ari-every 1 --budget-s 100 || exit 1
