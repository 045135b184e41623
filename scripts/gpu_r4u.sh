# Round 4: exact kernel with bank-spread default capacities (71 / 39): parity,
# probe, the LDS pass of the PMC; then the run-kernel phase timers (r4t).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "exact or dropin or c_abi" \
  > gpurun_out/r4u_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r4u_pytest.log; [ $rc -eq 0 ] || exit 1
for C in 2048 4096; do timeout -k 10 200 python scripts/exact_probe.py $C >> gpurun_out/r4u_exact.json 2>> gpurun_out/r4u_exact.log || exit 1; done
cat gpurun_out/r4u_exact.json
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU \
  -d gpurun_out/pmcx_r4u -o run --output-format csv -- python3 scripts/exact_probe.py 2048 > gpurun_out/pmcx_r4u.log 2>&1 &&
python3 - <<'PY'
import csv, glob
from collections import defaultdict
per = defaultdict(lambda: defaultdict(float))
for f in glob.glob("gpurun_out/pmcx_r4u/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mvc_exact_sweep_kernel" in r["Kernel_Name"]:
            per[r.get("Dispatch_Id", "")][r["Counter_Name"]] += float(r["Counter_Value"])
last = sorted(per, key=lambda k: int(k) if str(k).isdigit() else 0)[-1]
print(dict(per[last]))
PY
rm -rf gpurun_out/pmcx_r4u
bash scripts/gpu_r4t.sh
