"""Does a live GPU context in the parent slow a child's GPU work?  The bench
runs its extras as child processes of the process that measured the headline
(r4v: the New_Simulation chains leg at about half its stand-alone speed).
    python scripts/parent_ctx_probe.py [reset]
Runs bench.py --leg newsim_chains as a child after this process has set up
torch.cuda and a parallel sampler (closed again); with `reset`, the parent
also calls hipDeviceReset first."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multiview-clustering_amd")]
import torch  # noqa: E402

import mvc_amd  # noqa: E402
from mvc_amd import data  # noqa: E402

x = torch.ones(1024, device="cuda:0")
torch.cuda.synchronize()
y, _ = data.synthetic(200000, 4, 128, 64, seed=1)
s = mvc_amd.Sampler(y, seed=1, mode="parallel")
s.sweep(3)
s.synchronize()
s.close()
if len(sys.argv) > 1 and sys.argv[1] == "reset":
    import ctypes
    del x
    torch.cuda.empty_cache()
    rc = ctypes.CDLL("libamdhip64.so").hipDeviceReset()
    print("hipDeviceReset", rc, file=sys.stderr)
r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--leg", "newsim_chains"], capture_output=True, text=True)
print(json.dumps({"parent_ctx": True, "reset": len(sys.argv) > 1, "leg": json.loads(r.stdout.strip().splitlines()[-1])}))
