"""Cold-start probe: the reference initialisation (4 tables, 2 dishes per view,
multiview_gibbs.cpp:12-103) and the first sweeps of the parallel schedule,
sweep by sweep: wall time, tables, dish counts and the repair counters.

    python scripts/coldstart.py --config c2 --sweeps 5
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multiview-clustering_amd")]

import mvc_amd  # noqa: E402
from mvc_amd import data  # noqa: E402

CONFIGS = {"c2": (100_000, 2, 64, 16), "c4": (1_000_000, 4, 128, 64), "c4s": (200_000, 4, 128, 64),
           "ns": (1_000_000, 4, 1, 64)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--sweeps", type=int, default=5)
    ap.add_argument("--budget-s", type=float, default=120.0)
    ap.add_argument("--warm", action="store_true", help="start at the generating partition (bench.py warm_state)")
    ap.add_argument("--seed", type=int, default=7)
    a = ap.parse_args()
    N, V, D, K = CONFIGS[a.config]
    y, z = data.synthetic(N, V, D, K, seed=1999)
    s = mvc_amd.Sampler(y, seed=a.seed, mode="parallel")
    if a.warm:
        import bench
        s.set_state(*bench.warm_state(z, V, K))
    s.synchronize()
    t_all = time.perf_counter()
    for it in range(a.sweeps):
        t0 = time.perf_counter()
        s.sweep(1)
        s.synchronize()
        dt = time.perf_counter() - t0
        t, d, h = s.state()
        rec = {"sweep": it, "s": round(dt, 4), "T": int(d.shape[1]), "K": s.dish_counts().tolist(),
               "zpath": s.zpath(), **s.repair_stats(), "sigma_g": h["sigma_global"]}
        print(json.dumps(rec), flush=True)
        if time.perf_counter() - t_all > a.budget_s:
            break
    s.close()


if __name__ == "__main__":
    main()
