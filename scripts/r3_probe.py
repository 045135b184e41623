"""Round-3 probe: state shapes where the in-order repair carries the sweep,
and the New_Simulation.R call (N = 200, V = 5) timed in both schedules.

    python scripts/r3_probe.py shapes      # north-star literal warm + configs[1] cold: T, K_v, movers per sweep
    python scripts/r3_probe.py newsim M    # New_Simulation.R:123-133 shape, M sweeps, both modes
    python scripts/r3_probe.py ns1         # one warm literal sweep (the PMC target)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multiview-clustering_amd")]

import bench  # noqa: E402
import mvc_amd  # noqa: E402
from mvc_amd import data  # noqa: E402


def sweeps(s, k, tag):
    for it in range(k):
        t0 = time.perf_counter()
        s.sweep(1)
        s.synchronize()
        dt = time.perf_counter() - t0
        _, d, h = s.state()
        print(json.dumps({"tag": tag, "sweep": it, "s": round(dt, 4), "T": int(d.shape[1]),
                          "K": s.dish_counts().tolist(), **s.repair_stats(),
                          "sigma_g": round(h["sigma_global"], 4)}), flush=True)


def main():
    what = sys.argv[1]
    if what in ("shapes", "ns1"):
        N, V, D, K, _ = bench.CONFIGS["ns"]
        y, z = data.synthetic(N, V, D, K, seed=1999)
        s = mvc_amd.Sampler(y, seed=1999, mode="parallel")
        s.set_state(*bench.warm_state(z, V, K))
        sweeps(s, 1 if what == "ns1" else 3, "ns-warm")
        s.close()
    if what == "shapes":
        N, V, D, K, _ = bench.CONFIGS["c2"]
        y, _ = data.synthetic(N, V, D, K, seed=1999)
        s = mvc_amd.Sampler(y, seed=1999, mode="parallel")
        sweeps(s, 3, "c2-cold")
        s.close()
    if what == "newsim":
        M = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
        y, _ = data.new_simulation(1999)
        for mode in ("parallel", "exact"):
            t0 = time.perf_counter()
            r = mvc_amd.run_gibbs_cpp(y, M, M * 9 // 10, 1, seed=1999, mode=mode, quiet=True)
            dt = time.perf_counter() - t0
            print(json.dumps({"tag": "newsim", "mode": mode, "M": M, "s": round(dt, 3),
                              "sweeps_per_s": round(M / dt, 1), "saved": len(r["table_of"]),
                              "T_last": int(len(r["dish_of"][-1][0]))}), flush=True)


if __name__ == "__main__":
    main()
