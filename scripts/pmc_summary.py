"""Per-pass HBM traffic of the z-resample pass from rocprofv3 PMC CSVs.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE
under-reports wide streaming reads (MI355X_MICROARCH.md, HBM/rocprofv3
section); our loads are 8 B per lane (an uncalibrated width), so the factor is
calibrated on the lp producer's y stream, whose byte count is known exactly
(N * D * 8 per view launch)."""
import csv
import json
import sys
from collections import defaultdict

tag = sys.argv[1]
cfg = "c4"
N, V, D = 1_000_000, 4, 128


def per_kernel(counter):
    rows = list(csv.DictReader(open(f"gpurun_out/pmcz_{tag}_{counter.split('_')[0].lower()}/run_counter_collection.csv")))
    acc = defaultdict(list)
    for r in rows:
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]) * 1024.0)
    return acc


fetch = per_kernel("FETCH_SIZE")
write = per_kernel("WRITE_SIZE")
# one z pass = V producer launches + one draw launch; count passes by the draw
passes = max(1, sum(len(v) for k, v in fetch.items() if "zdraw" in k))
# calibration: every lpview launch streams N*D*8 bytes of y plus small tables
lp_fetch = [b for k, v in fetch.items() if "lpview" in k for b in v]
la_fetch = [b for k, v in fetch.items() if "lpall" in k for b in v]   # all-views producer: V views per launch
if la_fetch:
    factor = (N * D * 8 * V) / (sum(la_fetch) / len(la_fetch))
else:
    factor = (N * D * 8) / (sum(lp_fetch) / len(lp_fetch)) if lp_fetch else 1.0
fetch_pass = factor * sum(sum(v) for v in fetch.values()) / passes
write_pass = sum(sum(v) for v in write.values()) / passes
out = {cfg: {"bytes_per_pass": int(fetch_pass + write_pass), "fetch_bytes": int(fetch_pass),
             "write_bytes": int(write_pass), "fetch_factor": round(factor, 4),
             "algorithmic_bytes": N * (8 * V * D + 8), "source": f"profiles/pmcz_{tag}_*",
             "per_kernel_fetch": {k: factor * sum(v) / len(v) for k, v in fetch.items()},
             "per_kernel_write": {k: sum(v) / len(v) for k, v in write.items()}}}
print(json.dumps(out, indent=1))
