"""Per-kernel SQ/MFMA counter averages from a gpu_pmc_z.sh run (diagnostic)."""
import csv
import sys
from collections import defaultdict

tag = sys.argv[1]
for grp in ("sq", "mfma"):
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f"gpurun_out/pmcz_{tag}_{grp}/run_counter_collection.csv")):
        acc[r["Kernel_Name"].split("((")[0][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
