"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

The reference itself cannot be built here (Rcpp/R absent),
so these vectors pin the oracle (and, on the GPU box, the HIP sampler)
against regression; they are NOT reference outputs.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multiview-clustering_amd")]

from oracle import oracle as O  # noqa: E402
from mvc_amd import data  # noqa: E402

CASES = {
    # name: (y, M, burn, thin, seed, chain, mode)
    "exact_newsim": (lambda: data.new_simulation(1999)[0], 120, 0, 1, 1999, 0, O.EXACT),
    "exact_config1": (lambda: data.config1(1)[0], 60, 10, 2, 7, 3, O.EXACT),
    "parallel_newsim": (lambda: data.new_simulation(1999)[0], 40, 0, 1, 1999, 0, O.PARALLEL),
    "parallel_d4": (lambda: data.synthetic(600, 3, 4, 8, seed=5)[0], 12, 0, 1, 11, 1, O.PARALLEL),
}


def fixture(name):
    make, M, burn, thin, seed, chain, mode = CASES[name]
    y = np.asarray(make(), dtype=np.float64)
    r = O.run(y, M, burn, thin, seed, chain=chain, mode=mode, math=O.PORTABLE)
    S = len(r["table_of"])
    Tm = max(d.shape[1] for d in r["dish_of"])
    V = y.shape[0]
    dish = np.full((S, V, Tm), -1, dtype=np.int32)
    for s, d in enumerate(r["dish_of"]):
        dish[s, :, : d.shape[1]] = d
    return dict(y=y, M=M, burn=burn, thin=thin, seed=seed, chain=chain, mode=mode,
                table_of=np.stack(r["table_of"]).astype(np.int32), dish_of=dish,
                n_tables=np.array([d.shape[1] for d in r["dish_of"]], dtype=np.int32),
                alpha_v=r["alpha_v"], sigma_v=r["sigma_v"], tau_v=r["tau_v"],
                alpha_global=r["alpha_global"], sigma_global=r["sigma_global"],
                trace_T=r["trace_T"], trace_draws=r["trace_draws"])


if __name__ == "__main__":
    for name in CASES:
        f = fixture(name)
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **f)
        print(name, os.path.getsize(path), "bytes")
