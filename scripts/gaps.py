"""Idle gaps between consecutive kernels of the timed sweeps in a rocprofv3
kernel trace (tuning aid): python scripts/gaps.py <run_kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# the last 40% of the trace: timed sweeps (after data upload / warmup)
rows = rows[int(len(rows) * 0.6):]
gap = defaultdict(float)
cnt = defaultdict(int)
dur = defaultdict(float)
for a, b in zip(rows, rows[1:]):
    k = b["Kernel_Name"].split("(")[0].split("<")[0][-40:]
    gap[k] += (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
    cnt[k] += 1
    dur[k] += (int(b["End_Timestamp"]) - int(b["Start_Timestamp"])) / 1e3
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
print(f"span {span:.1f} us over {len(rows)} kernels; busy {sum(dur.values()):.1f} us, gaps {sum(gap.values()):.1f} us")
for k in sorted(gap, key=lambda k: -gap[k]):
    print(f"{k:42s} n={cnt[k]:4d} gap_before_avg={gap[k] / cnt[k]:7.2f} us dur_avg={dur[k] / cnt[k]:8.2f} us")
