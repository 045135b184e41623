"""Synthetic data generated on the device (mvc_sampler_create_synthetic) and
BASELINE configs[4] at its full size (N = 10M, V = 8, D = 256, K = 256:
164 GB of fp64 y, which fits the MI355X's HBM but not the host).

The full-size test checks, against the CPU where the CPU can hold the data:
  * the generating labels and the per-dish counts n_vk (exact integers);
  * S1 of whole dishes against host fp64 sums of the same rows (tolerance
    from the two summation orders: |dS1| <= 2 n eps sum|y|);
  * a warm sweep: every customer's phase-A draw of a 2,000-customer sample
    recomputed by the oracle from the device's statistics and those
    customers' rows (oracle.phase_a: the same conditional, bit for bit);
  * labels in range, every table non-empty, counts summing to N.
"""
import os
import time

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _progress(msg):
    """A line per phase under gpurun_out/ (a long GPU test stays visibly alive)."""
    root = os.environ.get("GRAFT_REPO_ROOT")
    if root:
        os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
        with open(os.path.join(root, "gpurun_out", "progress_test_synthetic.log"), "a") as f:
            f.write(f"{time.strftime('%H:%M:%S')} {msg}\n")


def _restate_labels(seed, n, K):
    """z_i of mvc_synth.hip: floor(K u), u from Philox{i, i >> 32, 0, 'MVSZ'}."""
    out = np.empty(n, dtype=np.int32)
    key = (seed & 0xFFFFFFFF, seed >> 32)
    for i in range(n):
        x, y_, _, _ = O.philox((i & 0xFFFFFFFF, i >> 32, 0, 0x4D56535A), key)
        u = (((y_ << 32 | x) >> 12) + 0.5) * 2.0 ** -52
        out[i] = min(int(u * K), K - 1)
    return out


def _restate_normals(seed, ctrs, tag):
    """R inversion normals from one Philox block each (mvc_synth.hip syn_normal)."""
    key = (seed & 0xFFFFFFFF, seed >> 32)
    u = np.empty(len(ctrs))
    for k, (c0, c1, c2) in enumerate(ctrs):
        x, y_, zz, w = O.philox((c0, c1, c2, tag), key)
        u1 = (((y_ << 32 | x) >> 12) + 0.5) * 2.0 ** -52
        u2 = (((w << 32 | zz) >> 12) + 0.5) * 2.0 ** -52
        u[k] = (float(int(134217728.0 * u1)) + u2) / 134217728.0
    return O.pm_qnorm(u)


def test_synthetic_generator_matches_restatement():
    """Labels and sampled values of the device generator equal the Python
    restatement of its Philox recipe bit for bit; a warm-started chain on the
    device data equals the oracle's chain on the same rows read back."""
    import mvc_amd
    N, V, D, K, seed, sd, mu_sd = 3000, 3, 16, 8, 77, 1.3, 3.0
    s, z = mvc_amd.Sampler.synthetic(N, V, D, K, data_seed=seed, sd=sd, mu_sd=mu_sd, seed=9)
    assert np.array_equal(z, _restate_labels(seed, N, K))
    rng = np.random.default_rng(1)
    for v in range(V):
        Kv = max(1, K >> v)
        idx = rng.choice(N, 20, replace=False)
        got = s.rows(v, idx)
        ds = rng.integers(0, D, 20)
        mu = mu_sd * _restate_normals(seed, [(v * K + int(z[i]) % Kv, int(d), 0) for i, d in zip(idx, ds)], 0x4D56534D)
        e = _restate_normals(seed, [(int(i), int(d), v) for i, d in zip(idx, ds)], 0x4D565359)
        assert np.array_equal(got[np.arange(20), ds], mu + sd * e), v
    y = np.stack([s.rows(v, np.arange(N)) for v in range(V)])
    T = int(z.max()) + 1
    dish = np.stack([np.arange(T) % max(1, K >> v) for v in range(V)]).astype(np.int32)
    hyper = np.array([1.69] * V + [1.0] * V + [0.5] * V + [1.0, 0.6])
    st = (z, dish, hyper)
    s.set_state(*st)
    ref = O.run(y, 3, 0, 1, seed=9, mode=O.PARALLEL, state=st)
    for it in range(3):
        s.sweep(1)
        t, d, h = s.state()
        assert np.array_equal(t, ref["table_of"][it]) and np.array_equal(d, ref["dish_of"][it]), it
        assert np.array_equal(h["tau_v"], ref["tau_v"][:, it]), it
    s.close()


def test_synthetic_handle_is_reproducible():
    """The same (data_seed, seed, chain) gives the same chain on every run:
    the generator's column sums (which seed tau_v, multiview_gibbs.cpp:78-94)
    are combined in a fixed order, so two handles agree bit for bit from
    their initial tau_v through a cold start."""
    import mvc_amd
    N, V, D, K = 100_000, 2, 8, 4
    runs = []
    for _ in range(2):
        s, z = mvc_amd.Sampler.synthetic(N, V, D, K, data_seed=11, seed=3)
        _, _, h0 = s.state()
        s.sweep(2)
        t, d, h = s.state()
        runs.append((h0["tau_v"].copy(), t, d, h["tau_v"].copy()))
        s.close()
    (a0, at, ad, ah), (b0, bt, bd, bh) = runs
    assert np.array_equal(a0, b0)
    assert np.array_equal(at, bt) and np.array_equal(ad, bd) and np.array_equal(ah, bh)


def test_config5_full_size_warm_sweep():
    """BASELINE configs[4] at N = 10M, V = 8, D = 256, K = 256 (the dish-block
    MFMA producer + the LDS-checkpoint draw; y generated on the device)."""
    import mvc_amd
    N, V, D, K, seed = 10_000_000, 8, 256, 256, 1999
    t0 = time.perf_counter()
    _progress("generating")
    s, z = mvc_amd.Sampler.synthetic(N, V, D, K, data_seed=seed, seed=seed)
    _progress(f"generated {time.perf_counter() - t0:.1f} s")
    T = int(z.max()) + 1
    assert T == K and np.array_equal(np.unique(z), np.arange(K))
    dish = np.stack([np.arange(T) % max(1, K >> v) for v in range(V)]).astype(np.int32)
    hyper = np.array([1.69] * V + [1.0] * V + [0.5] * V + [1.0, 0.6])
    s.set_state(z, dish, hyper)
    _progress(f"state set {time.perf_counter() - t0:.1f} s")
    stats = [s.stats(v) for v in range(V)]
    for v in range(V):
        Kv = max(1, K >> v)
        assert np.array_equal(stats[v]["n"], np.bincount(z % Kv, minlength=Kv)), v
    # S1 of whole dishes vs host sums of the same rows
    for v, c in ((0, 3), (1, 100)):
        Kv = max(1, K >> v)
        members = np.flatnonzero(z % Kv == c).astype(np.int32)
        rows = s.rows(v, members)
        host = rows.sum(axis=0)
        bound = 2.0 * members.size * np.finfo(float).eps * np.abs(rows).sum(axis=0)
        assert np.all(np.abs(stats[v]["S1"][c] - host) <= bound), (v, c)
        assert abs(stats[v]["S2"][c] - np.einsum("ij,ij->", rows, rows)) <= 2.0 * members.size * D * \
            np.finfo(float).eps * stats[v]["S2"][c]
    _progress(f"stats checked {time.perf_counter() - t0:.1f} s")
    ts = time.perf_counter()
    s.sweep(1)
    s.synchronize()
    sweep_s = time.perf_counter() - ts
    _progress(f"swept {sweep_s:.3f} s")
    t, d, h = s.state()
    rep = s.repair_stats()
    assert t.min() >= 0 and t.max() < d.shape[1]
    assert np.all(np.bincount(t, minlength=d.shape[1]) > 0)
    for v in range(V):
        assert s.stats(v)["n"].sum() == N
    assert s.zpath() & 64, "configs[4] runs the dish-block MFMA producer"
    # the device's phase-A conditional of sampled customers, recomputed on the CPU
    rng = np.random.default_rng(5)
    idx = np.sort(rng.choice(N, 2000, replace=False)).astype(np.int32)
    rows = np.stack([s.rows(v, idx) for v in range(V)], axis=1)        # [m][V][D]
    ch = O.phase_a(z, dish, hyper, stats, seed, 0, 0, idx, rows)
    if rep["moves"] == 0:
        assert np.array_equal(ch, t[idx])
    else:   # customers before the first mover keep their phase-A draw
        first = int(np.flatnonzero(t != z)[0]) if np.any(t != z) else N
        assert np.array_equal(ch[idx < first], z[idx[idx < first]])
    print(f"configs[4] N=10M: data+state {ts - t0:.1f} s, warm sweep {sweep_s:.3f} s, moves {rep['moves']}")
    _progress("done")
    s.close()
