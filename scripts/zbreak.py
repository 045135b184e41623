"""Timing breakdown of the z-resample kernel (MVC_Z_DEBUG skip flags).
Debug runs do NOT compute the spec; timing experiments only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multiview-clustering_amd")]
import bench  # noqa: E402
from mvc_amd import data  # noqa: E402
from mvc_amd.sampler import Sampler  # noqa: E402

N, V, D, K, _ = bench.CONFIGS[os.environ.get("ZB_CONFIG", "c4")]
y, z = data.synthetic(N, V, D, K, seed=1999)
st = bench.warm_state(z, V, K)
for flag in sys.argv[1:]:
    os.environ["MVC_Z_DEBUG"] = flag
    s = Sampler(y, seed=1999, mode="parallel", timing=True)
    s.set_state(*st)
    s.sweep(2)
    s.synchronize()
    s.reset_timers()
    t0 = time.perf_counter()
    s.sweep(10)
    s.synchronize()
    wall = (time.perf_counter() - t0) / 10 * 1e3
    ms, cnt = s.kernel_time("zresample")
    sw, _ = s.kernel_time("sweep")
    T = s.state()[1].shape[1]
    print(f"zdebug={flag} zresample {ms / cnt:.3f} ms  sweep(ev) {sw / 10:.3f} ms  wall {wall:.3f} ms  "
          f"T={T} K={s.dish_counts().tolist()} path={s.zpath()}", flush=True)
    s.close()
