"""Which bench leg slows the configs[1] cold-start leg that runs after it (probe)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multiview-clustering_amd")]
import bench  # noqa: E402


def cs(tag):
    r = bench.cold_start(1999, 0, sweeps=2)
    print(json.dumps({"after": tag, "cold": [x["s"] for x in r["sweeps"]]}), flush=True)


def main():
    import mvc_amd
    from mvc_amd import data
    cs("nothing")
    y, _ = data.new_simulation(1999)
    t0 = time.perf_counter()
    mvc_amd.run_gibbs_cpp(y, 1000, 500, 1, seed=1999, mode="parallel", n_chains=16, device=0, quiet=True)
    print(json.dumps({"leg": "newsim parallel 16 chains", "s": round(time.perf_counter() - t0, 2)}), flush=True)
    cs("newsim parallel 16 chains")
    t0 = time.perf_counter()
    mvc_amd.run_gibbs_cpp(y, 500, 250, 1, seed=1999, mode="exact", n_chains=256, device=0, quiet=True)
    print(json.dumps({"leg": "newsim exact 256 chains", "s": round(time.perf_counter() - t0, 2)}), flush=True)
    cs("newsim exact 256 chains")
    bench.gpu_chains_line("ns", 1999, 0)
    cs("literal 16 chains")


if __name__ == "__main__":
    main()
