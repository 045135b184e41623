"""Phase-A timing probe (configs[3] warm state): the z-resample pass alone
(mvc_sampler_phase_a: the state is unchanged, so timing-ablation builds of
the library -- MVC_ABL_* flags, scripts/build_variant.sh -- can run it) with
per-kernel HIP events.  Prints one JSON line: lp producer and draw ms."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multiview-clustering_amd")]
import bench  # noqa: E402
from mvc_amd import data  # noqa: E402
from mvc_amd.sampler import Sampler  # noqa: E402

cfg = os.environ.get("ZP_CONFIG", "c4")
reps = int(os.environ.get("ZP_REPS", "10"))
N, V, D, K, _ = bench.CONFIGS[cfg]
y, z = data.synthetic(N, V, D, K, seed=1999)
s = Sampler(y, seed=1999, mode="parallel", timing=True)
s.set_state(*bench.warm_state(z, V, K))
s.sweep(1)
s.synchronize()
ref = s.phase_a()
s.reset_timers()
for _ in range(reps):
    out = s.phase_a()
s.synchronize()
r = {"lib": os.environ.get("MVC_HIP_LIB", "default"), "config": cfg, "reps": reps}
for k in ("lp", "draw", "zresample"):
    ms, cnt = s.kernel_time(k)
    r[k] = round(ms / max(cnt, 1), 4)
r["choices_same"] = bool((out == ref).all())
s.close()
print(json.dumps(r), flush=True)
