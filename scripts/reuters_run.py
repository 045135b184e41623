"""BASELINE config 3: Reuters-21578 views (mvc_amd.reuters), K = 6 topics,
8 chains on one MI355X (concurrent, ChainSet), from the reference's cold
initialisation.  Prints one JSON line per sweep (seconds, tables per chain)
and, every --ari-every sweeps, the ARI (mcclust::arandi on the device) of
each chain's tables against the top-6 TOPICS of the scored documents.

    python scripts/reuters_run.py --sweeps 20 --chains 8
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multiview-clustering_amd")]


import numpy as np  # noqa: E402

import mvc_amd  # noqa: E402
from mvc_amd import reuters  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweeps", type=int, default=20)
    ap.add_argument("--chains", type=int, default=8)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--ari-every", type=int, default=5)
    ap.add_argument("--budget-s", type=float, default=150.0)
    ap.add_argument("--drop-topics", action="store_true",
                    help="zero the TOPICS columns of the third view (the ARI truth; mvc_amd.reuters)")
    ap.add_argument("--standardize", action="store_true",
                    help="every projected dimension centred and scaled to unit variance (mvc_amd.reuters.views)")
    ap.add_argument("--save", default=None, help="write every chain's state here (npz) at the end")
    ap.add_argument("--resume", default=None,
                    help="start every chain from a state --save wrote (the chains continue with fresh sweep "
                         "counters: a valid continuation of each chain, not the bitwise one)")
    a = ap.parse_args()
    y = reuters.views(drop_topics=a.drop_topics, standardize=a.standardize)
    lab, names, _ = reuters.topic_truth()
    sel = lab >= 0
    s = mvc_amd.Sampler(y, seed=a.seed, mode="parallel", n_chains=a.chains)
    start = 0
    if a.resume:
        st = np.load(a.resume)
        start = int(st["sweeps"])
        for c in range(a.chains):
            s.set_state(st[f"t{c}"], st[f"d{c}"], st[f"h{c}"], chain=c)
    s.synchronize()
    t_all = time.perf_counter()
    for it in range(a.sweeps):
        t0 = time.perf_counter()
        s.sweep(1)
        s.synchronize()
        dt = time.perf_counter() - t0
        rec = {"sweep": start + it, "s": round(dt, 4), "drop_topics": a.drop_topics, "standardize": a.standardize}
        Ts, aris, moves, taus = [], [], [], []
        for c in range(a.chains):
            t, d, h = s.state(chain=c)
            Ts.append(int(d.shape[1]))
            taus.append([round(float(x), 5) for x in h["tau_v"]])
            moves.append(s.repair_stats(chain=c)["moves"])
            if (it + 1) % a.ari_every == 0 or it == a.sweeps - 1:
                aris.append(round(float(mvc_amd.ari(t[sel], lab[sel])), 4))
        rec["T"] = Ts
        rec["moves"] = moves
        rec["tau_v_chain0"] = taus[0]
        if aris:
            rec["ari_top6"] = aris
        print(json.dumps(rec), flush=True)
        if time.perf_counter() - t_all > a.budget_s:
            break
    if a.save:
        out = {"sweeps": np.int64(start + it + 1)}
        for c in range(a.chains):
            t, d, h = s.state(chain=c)
            hv = np.concatenate([h["tau_v"], h["alpha_v"], h["sigma_v"], [h["alpha_global"], h["sigma_global"]]])
            out[f"t{c}"], out[f"d{c}"], out[f"h{c}"] = t, d, hv
        np.savez(a.save, **out)
    s.close()


if __name__ == "__main__":
    main()
