"""Time the reference's own caller shape (New_Simulation.R:123-133: N = 200,
V = 5) through mvc_run (run_gibbs_cpp): exact schedule with 1 / 256 / 1024 /
2048 chains per call and the parallel schedule with one chain; prints one
JSON line.  Run on the GPU box (scripts/gpu_r3y.sh)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multiview-clustering_amd"))
import mvc_amd  # noqa: E402
from mvc_amd import data  # noqa: E402

y, _ = data.new_simulation(1999)
out = {}
for mode, C, M in (("exact", 1, 2000), ("parallel", 1, 2000), ("exact", 256, 500), ("exact", 1024, 500),
                   ("exact", 1536, 500), ("exact", 2048, 500)):
    t0 = time.perf_counter()
    mvc_amd.run_gibbs_cpp(y, M, M // 2, 1, seed=1999, mode=mode, n_chains=C, quiet=True)
    dt = time.perf_counter() - t0
    out[f"{mode}_{C}"] = {"chains": C, "sweeps": M, "s": round(dt, 3), "chain_sweeps_per_s": round(C * M / dt, 1)}
    print(f"{mode} {C} chains: {C * M / dt:.1f} chain-sweeps/s", file=sys.stderr, flush=True)
# the same without mvc_run's sample bookkeeping: sweeps only
for mode, C, M in (("exact", 1, 2000), ("exact", 256, 500), ("exact", 1536, 500), ("exact", 2048, 500)):
    smp = mvc_amd.Sampler(y, seed=1999, mode=mode, n_chains=C)
    smp.sweep(2)
    smp.synchronize()
    t0 = time.perf_counter()
    smp.sweep(M)
    smp.synchronize()
    dt = time.perf_counter() - t0
    smp.close()
    out[f"{mode}_{C}_sweeps_only"] = {"chains": C, "sweeps": M, "s": round(dt, 3), "chain_sweeps_per_s": round(C * M / dt, 1)}
    print(f"{mode} {C} chains, sweeps only: {C * M / dt:.1f} chain-sweeps/s", file=sys.stderr, flush=True)
print(json.dumps(out))
