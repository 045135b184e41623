cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_reuters.py -x -v --timeout 250 --timeout-method thread -k "zpath2 or config5 or dish_block or reuters or capacity or config2 or golden" > gpurun_out/pt_zd.log 2>&1 || { tail -30 gpurun_out/pt_zd.log; exit 1; }
tail -2 gpurun_out/pt_zd.log
timeout -k 10 300 python -u bench.py --config c5s --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/zd_c5s.json 2> gpurun_out/zd_c5s.err || { tail gpurun_out/zd_c5s.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/zd_c5s.json').readline()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_sweep'], d['roofline']['achieved'], d['hbm']['lp_producer'], d['hbm']['draw'])"
