# Round 5: blocks per CU of the dish-block producer's narrow instances
# (configs[4] bench leg, MVC_BIG_BPC = 2 / 3 / 4), kernel summary at the default.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5x}
for b in 2 3 4; do
  MVC_BIG_BPC=$b timeout -k 10 300 python3 bench.py --leg configs4_full_gpu > gpurun_out/${TAG}_c5_bpc$b.json 2>&1 || exit 1
  echo "bpc $b: $(tail -1 gpurun_out/${TAG}_c5_bpc$b.json | cut -c1-330)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c5prof -o run --output-format csv -- \
  python3 bench.py --leg configs4_full_gpu > gpurun_out/${TAG}_c5prof.log 2>&1 || { echo "prof failed"; exit 1; }
find gpurun_out/${TAG}_c5prof -name "*kernel_trace.csv" -delete
