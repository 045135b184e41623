import os, sys, numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path[:0] = [ROOT, os.path.join(ROOT, "multiview-clustering_amd")]
import mvc_amd as m
from mvc_amd import data
from oracle import oracle as O
y, _ = data.new_simulation(1999)
M = int(sys.argv[1]) if len(sys.argv) > 1 else 60
ref = O.run(y, M, 0, 1, seed=1999, mode=O.PARALLEL)
s = m.Sampler(y, seed=1999, mode="parallel")
for it in range(M):
    s.sweep(1)
    t, d, h = s.state()
    if not np.array_equal(t, ref["table_of"][it]):
        bad = np.nonzero(t != ref["table_of"][it])[0]
        print("first diff at sweep", it, "zpath", s.zpath(), "T", d.shape, "customers", bad[:10], t[bad[:5]], ref["table_of"][it][bad[:5]])
        print("prev sweep zpath ok; tau", h["tau_v"], ref["tau_v"][:, it])
        break
else:
    print("all", M, "sweeps equal")
