"""The reference's own call (New_Simulation.R: N = 200, V = 5) through mvc_run
in the parallel schedule, for a kernel-trace profile: sweeps/s of the call
and the per-sweep repair counters of the last sweep."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multiview-clustering_amd")]
import mvc_amd  # noqa: E402
from mvc_amd import data  # noqa: E402

M = int(os.environ.get("NS_SWEEPS", "2000"))
mode = os.environ.get("NS_MODE", "parallel")
y, _ = data.new_simulation(1999)
mvc_amd.run_gibbs_cpp(y, 50, 49, 1, seed=1999, mode=mode, quiet=True)   # warm the runtime
t0 = time.perf_counter()
mvc_amd.run_gibbs_cpp(y, M, M - 1, 1, seed=1999, mode=mode, quiet=True)
dt = time.perf_counter() - t0
print(f"newsim {mode}: {M} sweeps in {dt:.3f} s = {M / dt:.1f} sweeps/s", flush=True)

# the repair's counters per sweep (rounds = run-kernel passes) on a handle
from mvc_amd.sampler import Sampler  # noqa: E402
s = Sampler(y, seed=1999, mode=mode)
s.sweep(300)
rows = []
for _ in range(8):
    s.sweep(1)
    rows.append(s.repair_stats())
s.close()
print("repair per sweep:", rows, flush=True)
