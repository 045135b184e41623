"""A/B kernel timing on the bench workload (tuning aid).

  python scripts/ab.py SPEC...   SPEC = [variant][:ENV=VAL[,ENV=VAL...]]
variant = build_variants/<variant>/libmvc_hip.so (scripts/build_variant.sh),
empty = the in-tree library.  Prints per-sweep ms of the timed kernels."""
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
N, V, D, K, _ = bench.CONFIGS[os.environ.get("AB_CONFIG", "c4")]
y, z = data.synthetic(N, V, D, K, seed=1999)
s = Sampler(y, seed=1999, mode="parallel", timing={{"0": False, "1": True, "coarse": "coarse"}}[os.environ.get("AB_TIMING", "1")])
s.set_state(*bench.warm_state(z, V, K))
s.sweep(2); s.synchronize(); s.reset_timers()
import time
t0 = time.perf_counter()
s.sweep(10); s.synchronize()
wall = (time.perf_counter() - t0) / 10 * 1e3
out = [sys.argv[1]]
for k in ("zresample", "lp", "draw", "commit", "stats", "hyper", "sweep"):
    ms, cnt = s.kernel_time(k)
    out.append(f"{{k}}={{ms / 10:.3f}}")
out.append(f"wall={{wall:.3f}}")
print(" ".join(out), flush=True)
'''.format(root=ROOT)
for spec in sys.argv[1:]:
    name, _, envs = spec.partition(":")
    env = dict(os.environ)
    if name:
        env["MVC_HIP_LIB"] = os.path.join(ROOT, "build_variants", name, "libmvc_hip.so")
    for kv in filter(None, envs.split(",")):
        k, v = kv.split("=")
        env[k] = v
    r = subprocess.run([sys.executable, "-c", CHILD, spec], env=env, timeout=300)
    if r.returncode != 0:
        sys.exit(r.returncode)
