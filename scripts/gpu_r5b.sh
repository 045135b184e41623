# Round 5: the slimmed all-views producer epilogue -- parity of the phase-A
# paths, then phase-A timing (default and ablations) and the bench line.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r5b}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "zpath2 or phase_a or config4 or mfma or warm_start or parallel_golden or generic or dish_block or last_customer" \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
for v in default abl_nostore abl_noepi; do
  if [ $v = default ]; then unset MVC_HIP_LIB; else export MVC_HIP_LIB=$PWD/build_variants/$v/libmvc_hip.so; fi
  timeout -k 10 200 python -u scripts/zprobe.py >> gpurun_out/${TAG}_zprobe.log 2>&1 || { echo "zprobe $v failed"; exit 1; }
done
unset MVC_HIP_LIB
cat gpurun_out/${TAG}_zprobe.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extras > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print(d['value'],d['roofline'],d['kernel_ms_per_sweep'])"
