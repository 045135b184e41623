"""Summary of scripts/gpu_pmc_run.sh / gpu_pmc_lane.sh: the run kernel's SQ counters summed over
its launches in one warm north-star-literal sweep, per repair iteration
(the iteration count is the run's own, from the probe log's first sweep)."""
import csv
import glob
import json
import sys
from collections import defaultdict

tag = sys.argv[1]
out = {"tag": tag, "kernel": "mvc_seq_run_kernel (every instance the sweep launched)", "counters": {}}
for grp in ("a", "b", "c", "d"):
    tot = defaultdict(float)
    launches = set()
    for f in glob.glob(f"gpurun_out/pmcr_{tag}_{grp}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "mvc_seq_run_kernel" not in r["Kernel_Name"] or (len(sys.argv) > 2 and sys.argv[2] not in r["Kernel_Name"]):
                continue
            launches.add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
    out["counters"].update({k: v for k, v in tot.items()})
    out[f"launches_{grp}"] = len(launches)
print(json.dumps(out, indent=1))
