"""North-star literal (N = 1M, V = 4, D = 1, K = 64) with C chains on one GPU
at once (ChainSet, DESIGN.md §7: the chain-batched repair by default;
MVC_PATH=chain_batch=0 one stream and host thread per chain, which needs
GPU_MAX_HW_QUEUES >= C): one sweep from the generating partition, aggregate
chain-sweeps/s.  Usage: python scripts/ns_chains.py C [C ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multiview-clustering_amd")]

import bench  # noqa: E402
from mvc_amd import data  # noqa: E402
from mvc_amd.sampler import Sampler  # noqa: E402


def main():
    N, V, D, K, desc = bench.CONFIGS["ns"]
    y, z = data.synthetic(N, V, D, K, seed=1999)
    st = bench.warm_state(z, V, K)
    for C in [int(a) for a in sys.argv[1:]] or [8]:
        s = Sampler(y, seed=1999, mode="parallel", n_chains=C, device=0)
        for c in range(C):
            s.set_state(*st, chain=c)
        s.synchronize()
        t0 = time.perf_counter()
        s.sweep(1)
        s.synchronize()
        dt = time.perf_counter() - t0
        s.close()
        print(json.dumps({"workload": desc.replace("1 chain/GPU", f"{C} chains on 1 GPU"), "chains": C,
                          "sweep_s": round(dt, 2), "chain_sweeps_per_s": round(C / dt, 3),
                          "batched": "chain_batch=0" not in os.environ.get("MVC_PATH", ""),
                          "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}), flush=True)


if __name__ == "__main__":
    main()
