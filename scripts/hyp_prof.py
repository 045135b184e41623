"""MH kernel phase marks (MVC_HYP_PROF build via MVC_HIP_LIB): configs[3]
warm, 8 sweeps; the kernel prints wall-clock ticks (100 MHz) at sweep 5."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multiview-clustering_amd")]
import bench  # noqa: E402
from mvc_amd import data  # noqa: E402
from mvc_amd.sampler import Sampler  # noqa: E402

cfg = os.environ.get("HP_CONFIG", "c4")
if cfg == "ns200":   # the reference's call shape (New_Simulation.R), cold
    y, _ = data.new_simulation(1999)
    s = Sampler(y, seed=1999, mode="parallel")
else:
    N, V, D, K, _ = bench.CONFIGS[cfg]
    y, z = data.synthetic(N, V, D, K, seed=1999)
    s = Sampler(y, seed=1999, mode="parallel")
    s.set_state(*bench.warm_state(z, V, K))
s.sweep(8)
s.synchronize()
s.close()
