"""Producer block-shape sweep (tuning aid): lp / draw / sweep ms per
(waves per block, blocks per CU) on the bench workload."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys
sys.path[:0] = [{root!r}, os.path.join({root!r}, "multiview-clustering_amd")]
import bench
from mvc_amd import data
from mvc_amd.sampler import Sampler
N, V, D, K, _ = bench.CONFIGS["c4"]
y, z = data.synthetic(N, V, D, K, seed=1999)
s = Sampler(y, seed=1999, mode="parallel", timing=True)
s.set_state(*bench.warm_state(z, V, K))
s.sweep(2); s.synchronize(); s.reset_timers()
s.sweep(10); s.synchronize()
out = [os.environ.get("MVC_LPV_WAVES"), os.environ.get("MVC_LPV_BPC")]
for k in ("lp", "draw", "sweep"):
    ms, cnt = s.kernel_time(k)
    out.append(f"{{k}}={{ms / 10:.3f}}")
print(" ".join(map(str, out)), flush=True)
'''.format(root=ROOT)
for spec in sys.argv[1:]:
    w, b = spec.split("x")
    env = dict(os.environ, MVC_LPV_WAVES=w, MVC_LPV_BPC=b)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, timeout=300)
    if r.returncode != 0:
        sys.exit(r.returncode)
