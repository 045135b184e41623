cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "shard" > gpurun_out/pt_shard.log 2>&1 || { tail -30 gpurun_out/pt_shard.log; exit 1; }
tail -2 gpurun_out/pt_shard.log
# two ranks sharing the one GPU (gloo): the --shard bench path end to end (timing meaningless)
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 WORLD_SIZE=2 LOCAL_RANK=0 MVC_BENCH_BACKEND=gloo
RANK=1 timeout -k 10 300 python -u bench.py --shard --steps 3 --warmup 1 --no-extras > gpurun_out/sb1.log 2>&1 &
P1=$!
RANK=0 timeout -k 10 300 python -u bench.py --shard --steps 3 --warmup 1 --no-extras > gpurun_out/sb0.log 2>&1
R0=$?
wait $P1; R1=$?
echo "rc $R0 $R1"; tail -3 gpurun_out/sb0.log; tail -3 gpurun_out/sb1.log
[ $R0 -eq 0 ] && [ $R1 -eq 0 ]
