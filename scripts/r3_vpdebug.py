"""Value prediction vs the plain lane-column loop on one chain: the first
customer whose table differs after sweep 0 (debug aid)."""
import os
import subprocess
import sys
import json

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multiview-clustering_amd")]


def run(vp, V, D, K, N, seed, sweeps):
    code = f"""
import os, sys, json, numpy as np
sys.path[:0] = [{ROOT!r}, os.path.join({ROOT!r}, 'multiview-clustering_amd')]
import mvc_amd
from mvc_amd import data
y, _ = data.synthetic({N}, {V}, {D}, {K}, seed={seed})
s = mvc_amd.Sampler(y, seed=17, mode='parallel')
out = []
for it in range({sweeps}):
    s.sweep(1)
    t, d, h = s.state()
    out.append(t.tolist())
print(json.dumps(out))
"""
    env = dict(os.environ, MVC_VP=vp, MVC_VP_STATS="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=200)
    sys.stderr.write(r.stderr[-3000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


for (V, D, K, N, seed) in [(5, 16, 6, 3000, 65), (5, 1, 6, 3000, 65), (3, 16, 6, 3000, 63)]:
    a = run("1", V, D, K, N, seed, 2)
    b = run("0", V, D, K, N, seed, 2)
    for it in range(len(a)):
        diff = [i for i in range(N) if a[it][i] != b[it][i]]
        print(json.dumps({"V": V, "D": D, "sweep": it, "ndiff": len(diff), "first": diff[:5]}), flush=True)
