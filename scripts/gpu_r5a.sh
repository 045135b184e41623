# Round 5 first GPU call: the new tests, phase-A timing ablations of the z
# pass, the z-pass PMC at HEAD and a kernel summary of the configs[4] leg.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_parity.py::test_last_customer_birth_with_poisoned_lds" \
  "tests/test_gpu_parity.py::test_run_n_devices_split_on_one_gpu" tests/test_bench_dist.py \
  > gpurun_out/r5a_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r5a_pytest.log; [ $rc -eq 0 ] || exit 1
for v in default abl_nostore abl_noepi abl_noview abl_nogather; do
  if [ $v = default ]; then unset MVC_HIP_LIB; else export MVC_HIP_LIB=$PWD/build_variants/$v/libmvc_hip.so; fi
  timeout -k 10 200 python -u scripts/zprobe.py >> gpurun_out/r5a_zprobe.log 2>&1 || { echo "zprobe $v failed"; exit 1; }
done
unset MVC_HIP_LIB
cat gpurun_out/r5a_zprobe.log
bash scripts/gpu_pmc_z.sh r5a || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5a_c5prof -o run --output-format csv -- \
  python3 bench.py --leg configs4_full_gpu > gpurun_out/r5a_c5prof.log 2>&1 || { echo "c5 prof failed"; exit 1; }
tail -1 gpurun_out/r5a_c5prof.log
find gpurun_out/r5a_c5prof -name "*kernel_trace.csv" -delete
find gpurun_out -path "*pmcz_r5a*" -name "*.csv" ! -name "*counter_collection*" -delete
echo done
