cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_reuters.py -x -v --timeout 250 --timeout-method thread -k "global_wide or reuters or repair_shapes or capacity or config2 or team" > gpurun_out/pt_wide.log 2>&1 || { tail -40 gpurun_out/pt_wide.log; exit 1; }
tail -2 gpurun_out/pt_wide.log
MVC_HIP_LIB=$GRAFT_REPO_ROOT/build_variants/runprof/libmvc_hip.so timeout -k 10 170 python -u scripts/reuters_run.py --sweeps 2 --chains 1 --ari-every 5 --budget-s 100 2>&1 | grep -v "^\[" || exit 1
timeout -k 10 170 python -u scripts/reuters_run.py --sweeps 3 --chains 8 --ari-every 3 --budget-s 100 || exit 1
