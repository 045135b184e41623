"""One New_Simulation.R-shaped call (N = 200, V = 5, New_Simulation.R:123-133)
through run_gibbs_cpp, parallel schedule, one chain (or argv[2] chains in
one call, MVC_CHAINS); prints sweeps/s.  For rocprofv3 kernel traces of the
reference's own call (scripts/gpu_r6.sh)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multiview-clustering_amd"))
import mvc_amd  # noqa: E402
from mvc_amd import data  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
C = int(sys.argv[2]) if len(sys.argv) > 2 else 1
y, _ = data.new_simulation(1999)
t0 = time.perf_counter()
mvc_amd.run_gibbs_cpp(y, M, M // 2, 1, seed=1999, mode="parallel", n_chains=C, quiet=True)
dt = time.perf_counter() - t0
print(f"newsim parallel {C} chain(s): {M} sweeps in {dt:.2f} s = {C * M / dt:.1f} chain-sweeps/s", flush=True)
