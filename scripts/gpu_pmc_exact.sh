#!/bin/bash
# PMC passes over the exact-schedule sweep kernel (scripts/exact_probe.py:
# New_Simulation shape, 2048 chains, two launches of 64 sweeps): one counter
# group per rocprofv3 run, kernel-trace only, CSV output.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-r4}
export TMPDIR=/tmp
run() {  # $1 = pass name, rest = counters
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmcx_${TAG}_$name -o run --output-format csv -- \
      python3 scripts/exact_probe.py 2048 > gpurun_out/pmcx_${TAG}_$name.log 2>&1 || { echo "pmc $name failed"; tail -5 gpurun_out/pmcx_${TAG}_$name.log; exit 1; }
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run b SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS SQ_INSTS_SMEM
run c SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC
run d SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_SALU SQ_WAVES
python3 - "$TAG" <<'PY'
import csv, glob, json, sys
from collections import defaultdict
tag = sys.argv[1]
out = {"tag": tag, "kernel": "mvc_exact_sweep_kernel (second launch)", "counters": {}}
for grp in ("a", "b", "c", "d"):
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"gpurun_out/pmcx_{tag}_{grp}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "mvc_exact_sweep_kernel" not in r["Kernel_Name"]:
                continue
            per[r.get("Dispatch_Id", r.get("Correlation_Id", ""))][r["Counter_Name"]] += float(r["Counter_Value"])
    if per:
        last = sorted(per, key=lambda k: int(k) if str(k).isdigit() else 0)[-1]
        out["counters"].update(per[last])
print(json.dumps(out, indent=1))
PY
rm -rf gpurun_out/pmcx_${TAG}_*/   # the raw CSVs (tens of MB); the summary above is what is kept
