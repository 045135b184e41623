"""Births and moves per sweep of the reference's own call at steady state
(N = 200, V = 5, New_Simulation.R:47-60; parallel schedule, one chain):
the repair counters of 300 sweeps after 1,000."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multiview-clustering_amd"))
import mvc_amd  # noqa: E402
from mvc_amd import data  # noqa: E402

y, _ = data.new_simulation(1999)
s = mvc_amd.Sampler(y, seed=1999, mode="parallel")
s.sweep(1000)
rec = []
for _ in range(300):
    s.sweep(1)
    r = s.repair_stats()
    rec.append((r["moves"], r["births"], r["rounds"], s.state()[1].shape[1]))
a = np.array(rec)
print("moves mean %.1f births mean %.2f (sweeps with a birth %.2f) rounds mean %.2f T mean %.1f max %d" % (
    a[:, 0].mean(), a[:, 1].mean(), (a[:, 1] > 0).mean(), a[:, 2].mean(), a[:, 3].mean(), a[:, 3].max()))
s.close()
