"""CPU tests of the oracle (test infrastructure, oracle/mvc_oracle.cpp).

The oracle is pinned by (a) the published Philox4x32-10 known-answer vectors
(Salmon et al., SC'11, Random123 kat_vectors), (b) accuracy of its portable
math against glibc / scipy, (c) the committed golden fixtures and (d) state
invariants.  Parity against the reference binary is unpinned (the reference
needs R/Rcpp, absent here).
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


# ------------------------------------------------------------------ Philox KATs
@pytest.mark.parametrize("ctr,key,expect", [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
])
def test_philox4x32_10_known_answers(ctr, key, expect):
    assert O.philox(ctr, key) == expect


def test_uniform_stream_properties():
    u = O.seq_uniforms(1999, 0, 0, 200000)
    assert np.all(u > 0.0) and np.all(u < 1.0)
    assert abs(u.mean() - 0.5) < 5e-3
    # counter-based: any window of the stream is reproducible on its own
    assert np.array_equal(O.seq_uniforms(1999, 0, 1234, 10), u[1234:1244])
    assert not np.array_equal(O.seq_uniforms(1999, 1, 0, 10), u[:10])   # chain id in the key


# ------------------------------------------------------------- portable math
def _ulps(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    ia = a.view(np.int64)
    ib = b.view(np.int64)
    ia = np.where(ia < 0, np.int64(-2**63) - ia, ia)
    ib = np.where(ib < 0, np.int64(-2**63) - ib, ib)
    return np.abs(ia - ib)


def test_pm_exp_log_within_one_ulp_of_glibc():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-700, 700, 100000), rng.uniform(-5, 5, 100000)])
    assert _ulps(O.pm_exp(x), np.exp(x)).max() <= 1
    y = np.concatenate([np.exp(rng.uniform(-700, 700, 100000)), rng.uniform(0.5, 2, 100000)])
    assert _ulps(O.pm_log(y), np.log(y)).max() <= 1
    assert O.pm_exp(np.array([-800.0]))[0] == 0.0
    assert np.isinf(O.pm_exp(np.array([800.0]))[0])
    assert O.pm_log(np.array([0.0]))[0] == -np.inf
    assert np.isnan(O.pm_log(np.array([-1.0]))[0])


def test_pm_lgamma_qnorm_accuracy():
    special = pytest.importorskip("scipy.special")
    stats = pytest.importorskip("scipy.stats")
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.uniform(1e-3, 30, 50000), rng.uniform(30, 1e6, 50000)])
    ref = special.gammaln(x)
    got = O.pm_lgamma(x)
    assert np.max(np.abs(got - ref) / np.maximum(1.0, np.abs(ref))) < 1e-13
    p = rng.uniform(1e-12, 1 - 1e-12, 50000)
    assert np.max(np.abs(O.pm_qnorm(p) - stats.norm.ppf(p))) < 1e-12


# ----------------------------------------------------------------- tree64 spec
def _butterfly64(x):
    s = np.zeros(64)
    s[: len(x)] = x
    h = 32
    while h >= 1:
        s[:h] = s[:h] + s[h:2 * h]
        h //= 2
    return s[0]


def _tree64(x):
    x = list(np.asarray(x, dtype=np.float64))
    if not x:
        return 0.0
    while True:
        x = [_butterfly64(x[c:c + 64]) for c in range(0, len(x), 64)]
        if len(x) == 1:
            return x[0]


@pytest.mark.parametrize("n", [1, 7, 64, 65, 300, 4097])
def test_tree64_sum_association(n):
    rng = np.random.default_rng(n)
    x = rng.exponential(size=n) * 10.0 ** rng.uniform(-8, 8, n)
    assert O.tree64_sum(x) == _tree64(x)


def test_tree64_select_picks_positive_leaf():
    rng = np.random.default_rng(3)
    for n in (1, 5, 64, 130):
        x = rng.exponential(size=n) * (rng.uniform(size=n) < 0.6)
        x[-1] = 1.0
        S = O.tree64_sum(x)
        for r in rng.uniform(0, S, 200):
            k = O.tree64_select(x, r)
            assert 0 <= k < n and x[k] > 0.0


# --------------------------------------------------------------- golden fixtures
GOLDENS = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz"))


@pytest.mark.parametrize("name", GOLDENS)
def test_oracle_reproduces_golden(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    r = O.run(z["y"], int(z["M"]), int(z["burn"]), int(z["thin"]), int(z["seed"]), chain=int(z["chain"]),
              mode=int(z["mode"]), math=O.PORTABLE)
    assert len(r["table_of"]) == z["table_of"].shape[0]
    for s, t in enumerate(r["table_of"]):
        assert np.array_equal(t, z["table_of"][s]), s
        T = int(z["n_tables"][s])
        assert np.array_equal(r["dish_of"][s], z["dish_of"][s][:, :T]), s
    for key in ("alpha_v", "sigma_v", "tau_v", "alpha_global", "sigma_global"):
        assert np.array_equal(r[key], z[key]), key
    assert np.array_equal(r["trace_T"], z["trace_T"])


# ---------------------------------------------------------------- invariants
def _check_state(table_of, dish_of, n):
    T = dish_of.shape[1]
    assert table_of.shape == (n,)
    assert table_of.min() >= 0 and table_of.max() < T
    assert np.all(np.bincount(table_of, minlength=T) > 0)        # no empty table survives a sweep
    assert np.all(dish_of >= 0)


@pytest.mark.parametrize("mode", [O.EXACT, O.PARALLEL])
def test_chain_invariants(mode):
    from mvc_amd import data
    y, _ = data.new_simulation(7)
    r = O.run(y, 30, 0, 1, 7, chain=2, mode=mode)
    n = y.shape[1]
    for t, d in zip(r["table_of"], r["dish_of"]):
        _check_state(t, d, n)
    assert np.all(r["alpha_global"] > 0) and np.all((r["sigma_global"] > 0) & (r["sigma_global"] < 1))
    assert np.all(r["tau_v"] > 0) and np.all((r["sigma_v"] > 0) & (r["sigma_v"] < 1))


def test_exact_schedule_libm_equals_portable_on_new_simulation():
    """The portable math is a restatement choice; on the reference's own
    script shape it must not change any decision of the exact schedule."""
    from mvc_amd import data
    y, _ = data.new_simulation(1999)
    a = O.run(y, 60, 0, 1, 1999, mode=O.EXACT, math=O.LIBM)
    b = O.run(y, 60, 0, 1, 1999, mode=O.EXACT, math=O.PORTABLE)
    assert all(np.array_equal(s, t) for s, t in zip(a["table_of"], b["table_of"]))


def test_burn_in_and_thin_select_saved_iterations():
    from mvc_amd import data
    y, _ = data.config1(2, n=120)
    full = O.run(y, 20, 0, 1, 5)
    thinned = O.run(y, 20, 5, 3, 5)
    keep = [it for it in range(20) if it >= 5 and (it - 5) % 3 == 0]   # multiview_gibbs.cpp:205
    assert len(thinned["table_of"]) == len(keep)
    for s, it in enumerate(keep):
        assert np.array_equal(thinned["table_of"][s], full["table_of"][it])


def test_warm_start_is_a_pure_function_of_the_state():
    from mvc_amd import data
    y, z = data.synthetic(800, 3, 4, 8, seed=3)
    T = int(z.max()) + 1
    dish = np.stack([np.arange(T) % (8 >> v) for v in range(3)]).astype(np.int32)
    hyper = np.array([1.69] * 3 + [1.0] * 3 + [0.5] * 3 + [1.0, 0.6])
    a = O.run(y, 4, 0, 1, 11, mode=O.PARALLEL, state=(z.astype(np.int32), dish, hyper))
    b = O.run(y, 4, 0, 1, 11, mode=O.PARALLEL, state=(z.astype(np.int32), dish, hyper))
    assert all(np.array_equal(s, t) for s, t in zip(a["table_of"], b["table_of"]))
    _check_state(a["table_of"][-1], a["dish_of"][-1], 800)


def test_phase_a_from_statistics_matches_the_sequential_sweep():
    """oracle.phase_a (the sweep-start conditional from given statistics and
    only the sampled rows; the CPU check of configs[4] at N = 10M) agrees
    with the oracle's own sweep: on a state with movers, every customer
    before the first mover draws its own table and the first mover does not."""
    from mvc_amd import data
    N, V, D, K = 2500, 3, 8, 6
    y, z = data.synthetic(N, V, D, K, seed=12)
    rng = np.random.default_rng(0)
    z = z.copy()
    flip = rng.choice(N, 200, replace=False)
    z[flip] = rng.integers(0, K, 200)              # a perturbed partition: customers move
    T = K
    dish = np.stack([np.arange(T) % max(1, K >> v) for v in range(V)]).astype(np.int32)
    hyper = np.array([1.69] * V + [1.0] * V + [0.5] * V + [1.0, 0.6])
    st = (z.astype(np.int32), dish, hyper)
    stats = O.run(y, 0, 0, 1, seed=3, mode=O.PARALLEL, state=st)["stats"]
    after = O.run(y, 1, 0, 1, seed=3, mode=O.PARALLEL, state=st)
    moved = np.flatnonzero(after["table_of"][0] != z)
    assert after["trace_moves"][0] > 0 and moved.size > 0
    first = int(moved[0])
    idx = np.arange(first + 1, dtype=np.int32)
    ch = O.phase_a(z, dish, hyper, stats, 3, 0, 0, idx, np.stack([y[:, i, :] for i in idx]))
    assert np.array_equal(ch[:first], z[:first]) and ch[first] != z[first]
