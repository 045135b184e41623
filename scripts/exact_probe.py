"""The exact schedule on the New_Simulation.R shape (N = 200, V = 5): C
chains, two launches of 64 sweeps each (the PMC target of
scripts/gpu_pmc_exact.sh; also prints the sweeps/s of the second launch).

    python scripts/exact_probe.py [C] [n] [warm] [timed]
    (n < 200: the first n customers; warm / timed sweeps, default 64 / 64)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multiview-clustering_amd")]
import mvc_amd  # noqa: E402
from mvc_amd import data  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
y, _ = data.new_simulation(1999)
if len(sys.argv) > 2:
    y = [v[: int(sys.argv[2])].copy() for v in y]
WARM = int(sys.argv[3]) if len(sys.argv) > 3 else 64
TIMED = int(sys.argv[4]) if len(sys.argv) > 4 else 64
s = mvc_amd.Sampler(y, seed=1999, mode="exact", n_chains=C)
s.sweep(WARM)
s.synchronize()
t0 = time.perf_counter()
s.sweep(TIMED)
s.synchronize()
dt = time.perf_counter() - t0
s.close()
print(json.dumps({"chains": C, "n": len(y[0]), "lib": os.path.basename(os.path.dirname(mvc_amd.lib()._name)),
                  "warm": WARM, "sweeps": TIMED, "s": round(dt, 4), "chain_sweeps_per_s": round(C * TIMED / dt, 1)}))
