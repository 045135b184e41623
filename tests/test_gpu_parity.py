"""GPU parity: libmvc_hip.so (through the C ABI) vs the CPU oracle.

Bar: bit-exact for every integer label and every fp64 hyperparameter, given
the same Philox seed (exact schedule = reference schedule; parallel schedule
= DESIGN.md §4 spec).  Run on an MI355X with ``pytest -m gpu``.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _path(monkeypatch, **kw):
    """Execution-path overrides of the library (MVC_PATH): one
    variable of key=value items, read when a sampler is created."""
    monkeypatch.setenv("MVC_PATH", ",".join(f"{k}={v}" for k, v in kw.items()))


def _mvc():
    import mvc_amd
    return mvc_amd


# ---------------------------------------------------------------- spec primitives
def test_device_exp_log_bitwise():
    m = _mvc()
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-745, 709.7, 200000), rng.uniform(-40, 40, 200000),
                        rng.uniform(-745.2, -707.5, 100000), rng.uniform(709.0, 709.79, 20000),
                        [0.0, -0.0, 1e-310, -1e-310, 709.78, -745.2, np.inf, -np.inf, np.nan]])
    assert np.array_equal(m.device_math("exp", x), O.pm_exp(x), equal_nan=True)
    assert np.array_equal(m.device_math("exp_sk", x), O.pm_exp(x), equal_nan=True)
    # the draw's exp: arguments of the form a - max (<= 0), never NaN
    xl = np.concatenate([x[(x <= 709.78) & ~np.isnan(x)], -rng.exponential(50.0, 200000),
                         rng.uniform(-746.0, -744.0, 100000), [-1e300, -5e5, -1100 * np.log(2)]])
    assert np.array_equal(m.device_math("exp_le0", xl), O.pm_exp(xl))
    y = np.concatenate([np.exp(rng.uniform(-700, 700, 200000)), rng.uniform(0.5, 2.0, 200000),
                        [0.0, 1.0, 2.0, 1e-320, np.inf, -1.0, np.nan]])
    assert np.array_equal(m.device_math("log", y), O.pm_log(y), equal_nan=True)
    y = np.concatenate([y, [-0.0, 5e-324, 2.2250738585072014e-308, 1.4142135623730951, 0.7071067811865476]])
    assert np.array_equal(m.device_math("log_nb", y), O.pm_log(y), equal_nan=True)


def test_device_lgamma_qnorm_sqrt_bitwise():
    m = _mvc()
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.uniform(1e-6, 30, 100000), rng.uniform(30, 2e6, 100000)])
    assert np.array_equal(m.device_math("lgamma", x), O.pm_lgamma(x))
    # the branch-free form (MH kernel): every recurrence length, tiny and huge arguments, the edges
    xb = np.concatenate([x, rng.uniform(0, 13, 100000), 10.0 ** rng.uniform(-300, 300, 20000),
                         [1e-320, 5e-324, 1.0, 2.0, 11.0, 11.999999999999998, 12.0, 12.000000000000002, 1e308]])
    assert np.array_equal(m.device_math("lgamma_nb", xb), O.pm_lgamma(xb))
    edge = np.array([0.0, -0.0, -1.0, np.inf, -np.inf, np.nan])
    assert np.array_equal(m.device_math("lgamma_nb", edge), m.device_math("lgamma", edge), equal_nan=True)
    p = np.concatenate([rng.uniform(0, 1, 100000), 10.0 ** rng.uniform(-30, -1, 10000)])
    assert np.array_equal(m.device_math("qnorm", p), O.pm_qnorm(p))
    s = rng.uniform(0, 1e6, 100000)
    assert np.array_equal(m.device_math("sqrt", s), np.sqrt(s))


def test_device_uniform_stream_bitwise():
    m = _mvc()
    for seed, chain, start in [(1999, 0, 0), (2**63 + 5, 7, 2**40 - 3)]:
        assert np.array_equal(m.device_seq_uniforms(seed, chain, start, 50000),
                              O.seq_uniforms(seed, chain, start, 50000))


def test_device_tree64_bitwise():
    m = _mvc()
    rng = np.random.default_rng(2)
    for n in (1, 5, 64, 65, 200, 4096):
        x = rng.exponential(size=(64, n)) * (rng.uniform(size=(64, n)) < 0.7)
        x[0] = 0.0
        x[0, -1] = 1.0
        sums_ref = np.array([O.tree64_sum(r) for r in x])
        r = rng.uniform(size=64) * sums_ref
        sums, sel = m.device_tree64(x, r)
        assert np.array_equal(sums, sums_ref)
        sel_ref = np.array([O.tree64_select(row, t) for row, t in zip(x, r)])
        assert np.array_equal(sel, sel_ref)
        pos = sums_ref > 0
        assert np.all(x[np.arange(64), sel][pos] > 0)


def test_mfma_f64_matches_fma_chain():
    """v_mfma_f64_16x16x4_f64 accumulation vs the k-ordered fma chain of the
    spec.  Records the bitwise agreement; bounded error."""
    m = _mvc()
    rng = np.random.default_rng(3)
    n, K, D = 64, 32, 128
    Y = rng.normal(0, 3, (n, D))
    S1 = rng.normal(0, 100, (K, D))
    G = m.device_gemm_check(Y, S1)
    ref = np.empty((n, K))
    for i in range(n):
        for j in range(K):
            acc = 0.0
            for d in range(D):
                acc = _fma(Y[i, d], S1[j, d], acc)
            ref[i, j] = acc
    frac = float(np.mean(G == ref))
    print(f"MFMA f64 bitwise agreement with fma chain: {frac:.6f}")
    assert np.allclose(G, ref, rtol=1e-12, atol=1e-9)


def _fma(a, b, c):
    from fractions import Fraction
    return float(Fraction(a) * Fraction(b) + Fraction(c))


# ---------------------------------------------------------------- exact schedule
def _compare(gpu, ref):
    assert len(gpu["table_of"]) == len(ref["table_of"])
    for s, (a, b) in enumerate(zip(gpu["table_of"], ref["table_of"])):
        assert np.array_equal(a, b), f"table_of differs at saved sample {s}"
    for s, (a, b) in enumerate(zip(gpu["dish_of"], ref["dish_of"])):
        assert np.array_equal(np.stack(a), np.asarray(b)), f"dish_of differs at saved sample {s}"
    for k in ("alpha_v", "sigma_v", "tau_v"):
        assert np.array_equal(np.stack(gpu[k]), ref[k]), k
    for k in ("alpha_global", "sigma_global"):
        assert np.array_equal(gpu[k], ref[k]), k


def _golden(name):
    f = np.load(os.path.join(GOLDEN, name + ".npz"))
    S = f["table_of"].shape[0]
    return f, {
        "table_of": list(f["table_of"]),
        "dish_of": [f["dish_of"][s, :, : f["n_tables"][s]] for s in range(S)],
        "alpha_v": f["alpha_v"], "sigma_v": f["sigma_v"], "tau_v": f["tau_v"],
        "alpha_global": f["alpha_global"], "sigma_global": f["sigma_global"],
    }


@pytest.mark.parametrize("name", ["exact_newsim", "exact_config1"])
def test_exact_golden(name):
    m = _mvc()
    f, ref = _golden(name)
    gpu = m.run_gibbs_cpp(f["y"], int(f["M"]), int(f["burn"]), int(f["thin"]), seed=int(f["seed"]),
                          mode="exact", first_chain=int(f["chain"]), quiet=True)
    _compare(gpu, ref)


def test_exact_many_chains_vs_live_oracle():
    m = _mvc()
    from mvc_amd import data
    y, _ = data.new_simulation(7)
    gpus = m.run_gibbs_cpp(y, 60, 20, 3, seed=42, mode="exact", n_chains=4, quiet=True)
    for c, g in enumerate(gpus):
        ref = O.run(y, 60, 20, 3, seed=42, chain=c, mode=O.EXACT, math=O.PORTABLE)
        _compare(g, ref)


def test_exact_run_many_chains_threaded_samples():
    """mvc_run with 256 chains: the saved samples are emitted on several host
    threads (one range of chains each); chains spread over the range are
    bitwise the oracle's, samples in order."""
    m = _mvc()
    from mvc_amd import data
    y, _ = data.new_simulation(5)
    gpus = m.run_gibbs_cpp(y, 8, 2, 2, seed=21, mode="exact", n_chains=256, quiet=True)
    assert len(gpus) == 256
    for c in (0, 37, 128, 255):
        ref = O.run(y, 8, 2, 2, seed=21, chain=c, mode=O.EXACT, math=O.PORTABLE)
        _compare(gpus[c], ref)


@pytest.mark.parametrize("mode", ["0", "1", "2"])
def test_exact_storage_modes(mode, monkeypatch):
    """The sweep kernel's three storage instances (every chain array in global
    memory / all but z in LDS / all in LDS; MVC_PATH exact_lds caps the one the
    sizes allow) give the oracle's chain through New_Simulation's cold
    transient (T ~ 170 of n = 200)."""
    _path(monkeypatch, exact_lds=mode)
    m = _mvc()
    from mvc_amd import data
    y, _ = data.new_simulation(11)
    gpus = m.run_gibbs_cpp(y, 40, 10, 3, seed=9, mode="exact", n_chains=3, quiet=True)
    for c, g in enumerate(gpus):
        ref = O.run(y, 40, 10, 3, seed=9, chain=c, mode=O.EXACT, math=O.PORTABLE)
        _compare(g, ref)


def test_exact_capacity_growth():
    """Tiny initial capacities force the overflow -> regrow -> resume path."""
    m = _mvc()
    from mvc_amd import data
    y, _ = data.config1(3, n=300)
    s = m.Sampler(y, seed=5, mode="exact", table_cap=8, dish_cap=4)
    ref = O.run(y, 15, 0, 1, seed=5, mode=O.EXACT, math=O.PORTABLE)
    for it in range(15):
        s.sweep(1)
        t, d, h = s.state()
        assert np.array_equal(t, ref["table_of"][it]), it
        assert np.array_equal(d, ref["dish_of"][it]), it
        assert h["alpha_global"] == ref["alpha_global"][it]
    s.close()


# ---------------------------------------------------------------- parallel schedule
@pytest.mark.parametrize("name", ["parallel_newsim", "parallel_d4"])
def test_parallel_golden(name):
    m = _mvc()
    f, ref = _golden(name)
    gpu = m.run_gibbs_cpp(f["y"], int(f["M"]), int(f["burn"]), int(f["thin"]), seed=int(f["seed"]),
                          mode="parallel", first_chain=int(f["chain"]), quiet=True)
    _compare(gpu, ref)


def test_parallel_vs_live_oracle_d1():
    m = _mvc()
    from mvc_amd import data
    y, _ = data.config1(11, n=2000)
    gpu = m.run_gibbs_cpp(y, 15, 0, 1, seed=3, mode="parallel", quiet=True)
    ref = O.run(y, 15, 0, 1, seed=3, mode=O.PARALLEL)
    _compare(gpu, ref)


def test_parallel_multichunk_stats():
    """n > stats chunk (4096): exercises the chunked rebuild order."""
    m = _mvc()
    from mvc_amd import data
    y, _ = data.synthetic(9000, 2, 2, 4, seed=8)
    gpu = m.run_gibbs_cpp(y, 4, 0, 1, seed=9, mode="parallel", quiet=True)
    ref = O.run(y, 4, 0, 1, seed=9, mode=O.PARALLEL)
    _compare(gpu, ref)


def test_dropin_output_shape():
    m = _mvc()
    from mvc_amd import data
    y, labels = data.new_simulation(1999)
    res = m.run_gibbs_cpp(list(y), 30, 20, 1, seed=1999, quiet=True)
    assert set(res) == {"table_of", "dish_of", "loglik", "alpha_v", "sigma_v", "tau_v", "alpha_global",
                        "sigma_global"}
    assert len(res["table_of"]) == 10 and len(res["dish_of"]) == 10
    assert len(res["alpha_v"]) == 5 and len(res["alpha_v"][0]) == 10
    assert res["loglik"].size == 0
    cl = m.get_final_clusters(res)
    assert cl.shape == (200, 5)


def test_parallel_capacity_growth():
    """Tiny initial capacities (16 tables, 15 dishes per view): the cold start
    of New_Simulation.R's shape opens ~70 tables in its first sweeps, so the
    repair's births overflow and every chain is grown and resumed (oracle:
    unbounded, multiview_utils.cpp:209-216, 251-258); the chain is unchanged."""
    m = _mvc()
    from mvc_amd import data
    y, _ = data.new_simulation(1999)
    s = m.Sampler(y, seed=5, mode="parallel", table_cap=16, dish_cap=15)
    ref = O.run(y, 12, 0, 1, seed=5, mode=O.PARALLEL)
    grew = False
    for it in range(12):
        s.sweep(1)
        t, d, h = s.state()
        grew |= d.shape[1] > 16
        assert np.array_equal(t, ref["table_of"][it]), it
        assert np.array_equal(d, ref["dish_of"][it]), it
        assert h["alpha_global"] == ref["alpha_global"][it]
    assert grew
    s.close()


def _check_sweeps(s, ref, sweeps, stats=True):
    for it in range(sweeps):
        s.sweep(1)
        t, d, h = s.state()
        assert np.array_equal(t, ref["table_of"][it]), it
        assert np.array_equal(d, ref["dish_of"][it]), it
        assert np.array_equal(h["tau_v"], ref["tau_v"][:, it]), it
        assert h["sigma_global"] == ref["sigma_global"][it], it
    if stats:
        for v in range(len(ref["stats"])):
            g, r = s.stats(v), ref["stats"][v]
            assert np.array_equal(g["n"], r["n"]) and np.array_equal(g["S1"], r["S1"]), v
            assert np.array_equal(g["S2"], r["S2"]), v


def test_config2_full_size_cold_and_warm():
    """BASELINE configs[1] at its full size (N = 100k, V = 2, D = 64, K = 16):
    3 sweeps from the reference initialisation (thousands of movers per sweep:
    the in-order repair carries the sweep) and 3 warm sweeps, bitwise."""
    m = _mvc()
    from mvc_amd import data
    N, V, D, K = 100_000, 2, 64, 16
    y, z = data.synthetic(N, V, D, K, seed=1999)
    s = m.Sampler(y, seed=11, mode="parallel")
    ref = O.run(y, 3, 0, 1, seed=11, mode=O.PARALLEL)
    _check_sweeps(s, ref, 3)
    assert s.repair_stats()["moves"] == ref["trace_moves"][-1]
    s.close()
    st = _warm_state(z, V, K)
    s = m.Sampler(y, seed=11, mode="parallel")   # fresh handle: sweep counter 0, like the oracle
    s.set_state(*st)
    ref = O.run(y, 3, 0, 1, seed=11, mode=O.PARALLEL, state=st)
    _check_sweeps(s, ref, 3)
    s.close()


def test_config4_full_size_warm_sweep():
    """BASELINE configs[3] shard at its full size (N = 1M, V = 4, D = 128,
    K = 64): one warm sweep of the benchmarked path, bitwise vs the oracle."""
    m = _mvc()
    from mvc_amd import data
    N, V, D, K = 1_000_000, 4, 128, 64
    y, z = data.synthetic(N, V, D, K, seed=1999)
    st = _warm_state(z, V, K)
    s = m.Sampler(y, seed=1999, mode="parallel")
    s.set_state(*st)
    ref = O.run(y, 1, 0, 1, seed=1999, mode=O.PARALLEL, state=st)
    _check_sweeps(s, ref, 1)
    assert s.zpath() & 2   # the MFMA producer
    s.close()


def test_config5_shape_reduced_n():
    """BASELINE configs[4]'s shape (V = 8, D = 256, K = 256 generating
    clusters: K_v = 256 ... 2) at N = 20k, warm start, bitwise."""
    m = _mvc()
    from mvc_amd import data
    N, V, D, K = 20_000, 8, 256, 256
    y, z = data.synthetic(N, V, D, K, seed=5)
    st = _warm_state(z, V, K)
    s = m.Sampler(y, seed=3, mode="parallel")
    s.set_state(*st)
    ref = O.run(y, 2, 0, 1, seed=3, mode=O.PARALLEL, state=st)
    _check_sweeps(s, ref, 2)
    s.close()


# ---------------------------------------------------------------- MFMA path, warm start
def _warm_state(z, V, K):
    from mvc_amd import data  # noqa: F401
    T = int(z.max()) + 1
    dish = np.stack([np.arange(T) % max(1, K // (2 ** v)) for v in range(V)]).astype(np.int32)
    hyper = np.array([1.69] * V + [1.0] * V + [0.5] * V + [1.0, 0.6])
    return z.astype(np.int32), dish, hyper


@pytest.mark.parametrize("D", [16, 32])
def test_parallel_mfma_path_cold(D):
    m = _mvc()
    from mvc_amd import data
    y, _ = data.synthetic(1200, 3, D, 8, seed=D)
    gpu = m.run_gibbs_cpp(y, 6, 0, 1, seed=21, mode="parallel", quiet=True)
    ref = O.run(y, 6, 0, 1, seed=21, mode=O.PARALLEL)
    _compare(gpu, ref)


@pytest.mark.parametrize("D", [1, 4, 64])
def test_parallel_warm_start(D):
    m = _mvc()
    from mvc_amd import data
    V, K = 4, 16
    y, z = data.synthetic(3000, V, D, K, seed=100 + D)
    st = _warm_state(z, V, K)
    s = m.Sampler(y, seed=77, mode="parallel")
    s.set_state(*st)
    ref = O.run(y, 5, 0, 1, seed=77, mode=O.PARALLEL, state=st)
    for it in range(5):
        s.sweep(1)
        t, d, h = s.state()
        assert np.array_equal(t, ref["table_of"][it]), it
        assert np.array_equal(d, ref["dish_of"][it]), it
        assert np.array_equal(h["tau_v"], ref["tau_v"][:, it]), it
        assert h["sigma_global"] == ref["sigma_global"][it]
    s.close()


def _run_path(m, y, st, seed, sweeps, path, monkeypatch, draw="reg", expect_reg=None):
    """Run `sweeps` warm-started sweeps forcing the lp producer (0 generic,
    2 MFMA) and the phase-1 kernels ("reg" lp buffer + register draw, "lds"
    lp buffer + checkpoint draw; "-perview" one producer launch per view);
    check the path taken on the first sweep."""
    _path(monkeypatch, generic="1" if path == 0 else "0", zdraw=draw.replace("-perview", ""),
          lpall="0" if draw.endswith("-perview") else "1")
    draw = draw.replace("-perview", "")
    s = m.Sampler(y, seed=seed, mode="parallel")
    s.set_state(*st)
    states = []
    for it in range(sweeps):
        s.sweep(1)
        if it == 0:          # later sweeps may leave the path's limits (births)
            zp = s.zpath()
            assert zp & 3 == path
            assert bool(zp & 4) == ((draw == "reg") if expect_reg is None else expect_reg)
            if draw.startswith("row"):
                assert zp & 128
            elif draw == "lds":
                assert not zp & 128
        states.append(s.state())
    s.close()
    return states


def test_mfma_and_generic_paths_identical(monkeypatch):
    m = _mvc()
    from mvc_amd import data
    V, K, D = 3, 8, 32
    y, z = data.synthetic(2000, V, D, K, seed=5)
    st = _warm_state(z, V, K)
    out = [_run_path(m, y, st, 9, 3, p, monkeypatch) for p in (0, 2)]
    for a in out[1:]:
        for sa, sb in zip(out[0], a):
            assert np.array_equal(sa[0], sb[0])
            assert np.array_equal(sa[1], sb[1])
            assert np.array_equal(sa[2]["tau_v"], sb[2]["tau_v"])


# MFMA lp producer (path 2): ragged tiles (n % 16 != 0), fewer tiles than
# waves, D not a multiple of 16 (zero-padded k-steps), T > 64, K_v of 64;
# phase 1 as lp buffer + register draw (T <= 64, K_v <= 64) or lp buffer +
# LDS checkpoint draw (any T), the all-views producer or one launch per view
ZPATH_SHAPES = [(3001, 4, 64, 16, 16), (50, 2, 20, 4, 4), (4000, 3, 32, 64, 96), (2500, 2, 128, 64, 64),
                (5000, 3, 32, 32, 200), (6000, 2, 16, 64, 300),
                (1500, 3, 16, 32, 40), (2000, 2, 24, 8, 24), (4100, 4, 128, 64, 64), (777, 1, 32, 16, 16)]


@pytest.mark.parametrize("draw", ["reg", "lds", "reg-perview", "row", "row-global"])
@pytest.mark.parametrize("n,V,D,K,T", ZPATH_SHAPES)
def test_zpath2_vs_oracle(n, V, D, K, T, draw, monkeypatch):
    m = _mvc()
    from mvc_amd import data
    y, z = data.synthetic(n, V, D, T, seed=n + D)
    uniq, table_of = np.unique(z, return_inverse=True)   # generating partition
    table_of = table_of.astype(np.int32)
    T = uniq.size
    dish = np.stack([np.arange(T) % max(1, K // (2 ** v)) for v in range(V)]).astype(np.int32)
    hyper = np.array([1.69] * V + [1.0] * V + [0.5] * V + [1.0, 0.6])
    st = (table_of, dish, hyper)
    gpu = _run_path(m, y, st, 31, 3, 2, monkeypatch, draw=draw, expect_reg=(draw.startswith("reg") and T <= 64))
    ref = O.run(y, 3, 0, 1, seed=31, mode=O.PARALLEL, state=st)
    for it in range(3):
        t, d, h = gpu[it]
        assert np.array_equal(t, ref["table_of"][it]), it
        assert np.array_equal(d, ref["dish_of"][it]), it
        assert np.array_equal(h["tau_v"], ref["tau_v"][:, it]), it
        assert h["sigma_global"] == ref["sigma_global"][it]


def test_many_views_row_draw_gate(monkeypatch):
    """More than 16 views with 64 < T <= 512: the row draw keeps one view per
    lane of a customer's 16-lane row, so it must not be selected (even under
    MVC_PATH zdraw=row); the checkpoint draw runs and the chain is bitwise the
    oracle's."""
    m = _mvc()
    from mvc_amd import data
    V, K = 18, 8
    y, z = data.synthetic(1200, V, 16, 96, seed=77)
    uniq, table_of = np.unique(z, return_inverse=True)
    table_of = table_of.astype(np.int32)
    T = uniq.size
    assert 64 < T <= 512
    dish = np.stack([np.arange(T) % max(1, K // (2 ** min(v, 3))) for v in range(V)]).astype(np.int32)
    hyper = np.array([1.69] * V + [1.0] * V + [0.5] * V + [1.0, 0.6])
    st = (table_of, dish, hyper)
    _path(monkeypatch, zdraw="row")
    s = m.Sampler(y, seed=41, mode="parallel")
    s.set_state(*st)
    ref = O.run(y, 2, 0, 1, seed=41, mode=O.PARALLEL, state=st)
    for it in range(2):
        s.sweep(1)
        if it == 0:
            assert not s.zpath() & 128
        t, d, h = s.state()
        assert np.array_equal(t, ref["table_of"][it]), it
        assert np.array_equal(d, ref["dish_of"][it]), it
    s.close()


# Phase A alone (mvc_sampler_phase_a) against the oracle's phase-A
# conditional: ragged tile groups (n % 64 != 0), fewer tiles than waves,
# T <= 16 / 64, the bench's dish pattern (64, 32, 16, 8) at D = 128 and
# configs[1]'s (16, 8) at D = 64, up to the bench's full N.
PHASE_A_SHAPES = [(4100, 4, 128, 64, 64), (3001, 2, 64, 16, 16), (70001, 4, 128, 64, 64), (777, 2, 64, 16, 16),
                  (300001, 2, 64, 16, 16), (1_000_000, 4, 128, 64, 64)]


@pytest.mark.parametrize("n,V,D,K,T", PHASE_A_SHAPES)
def test_phase_a_vs_oracle(n, V, D, K, T):
    """Every customer up to 300k, a sample of 40k (incl. the first and last
    tiles) beyond; from the state after one sweep (statistics kept
    incrementally)."""
    m = _mvc()
    from mvc_amd import data
    y, z = data.synthetic(n, V, D, T, seed=n + D + 2)
    uniq, table_of = np.unique(z, return_inverse=True)
    table_of = table_of.astype(np.int32)
    T = uniq.size
    dish = np.stack([np.arange(T) % max(1, K // (2 ** v)) for v in range(V)]).astype(np.int32)
    hyper = np.array([1.69] * V + [1.0] * V + [0.5] * V + [1.0, 0.6])
    if n <= 300_001:
        idx = np.arange(n, dtype=np.int32)
    else:
        rng = np.random.default_rng(n)
        idx = np.unique(np.concatenate([np.arange(256), np.arange(n - 256, n),
                                        rng.choice(n, 40_000, replace=False)])).astype(np.int32)
    s = m.Sampler(y, seed=41, mode="parallel")
    s.set_state(table_of, dish, hyper)
    s.sweep(1)                            # phase A of sweep 1
    t1, d1, h1 = s.state()
    ch = s.phase_a()
    assert s.zpath() & 4                  # the register draw
    stats = [s.stats(v) for v in range(V)]
    rows = np.ascontiguousarray(np.transpose(y[:, idx, :], (1, 0, 2)))
    ref = O.phase_a(t1, d1, np.concatenate([h1["tau_v"], h1["alpha_v"], h1["sigma_v"],
                                            [h1["alpha_global"], h1["sigma_global"]]]), stats, 41, 0, 1, idx, rows)
    assert np.array_equal(ch[idx], ref), int(np.sum(ch[idx] != ref))
    # the pass changed nothing: a sweep now equals a sweep without the call
    s2 = m.Sampler(y, seed=41, mode="parallel")
    s2.set_state(table_of, dish, hyper)
    s2.sweep(1)
    s.sweep(1)
    s2.sweep(1)
    assert np.array_equal(s.state()[0], s2.state()[0])
    s.close()
    s2.close()


def test_exact_warm_start():
    m = _mvc()
    from mvc_amd import data
    y, z = data.config1(4, n=400)
    dish = np.array([[0, 1, 2], [0, 1, 0]], dtype=np.int32)
    hyper = np.array([1.69, 1.69, 1.0, 1.0, 0.5, 0.5, 1.0, 0.6])
    s = m.Sampler(y, seed=8, mode="exact")
    s.set_state(z.astype(np.int32), dish, hyper)
    ref = O.run(y, 6, 0, 1, seed=8, mode=O.EXACT, math=O.PORTABLE, state=(z.astype(np.int32), dish, hyper))
    for it in range(6):
        s.sweep(1)
        t, d, h = s.state()
        assert np.array_equal(t, ref["table_of"][it]), it
        assert np.array_equal(d, ref["dish_of"][it]), it
        assert h["alpha_global"] == ref["alpha_global"][it]
    s.close()


# ------------------------------------------------------ C-ABI from plain C (dlopen)
def test_c_abi_example_matches_python_path(tmp_path):
    """examples/mvc_abi_example.c drives libmvc_hip.so through dlopen/dlsym
    only (the Rcpp drop-in's path); its result equals the ctypes path."""
    import subprocess
    m = _mvc()
    from mvc_amd import data
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = tmp_path / "mvc_abi_example"
    subprocess.run(["gcc", "-O2", "-I", os.path.join(root, "include"), "-o", str(exe),
                    os.path.join(root, "examples", "mvc_abi_example.c"), "-ldl"], check=True)
    y, _ = data.new_simulation(11)
    V, n = y.shape
    M, burn, thin, mode, seed = 40, 10, 2, 0, 4242
    inp = tmp_path / "in.bin"
    with open(inp, "wb") as f:
        np.array([n, V, 1, M, burn, thin, mode], dtype=np.int32).tofile(f)
        np.array([seed], dtype=np.uint64).tofile(f)
        np.ascontiguousarray(y, dtype=np.float64).tofile(f)
    out = tmp_path / "out.bin"
    subprocess.run([str(exe), m.LIB_PATH, str(inp), str(out)], check=True, timeout=300)
    raw = open(out, "rb").read()
    S, T = np.frombuffer(raw[:8], dtype=np.int32)
    tab = np.frombuffer(raw[8:8 + 4 * n], dtype=np.int32)
    dish = np.frombuffer(raw[8 + 4 * n:8 + 4 * n + 4 * V * T], dtype=np.int32).reshape(V, T)
    ag = np.frombuffer(raw[8 + 4 * n + 4 * V * T:], dtype=np.float64)[:S]
    ref = m.run_gibbs_cpp(y, M, burn, thin, seed=seed, mode="exact", quiet=True)
    assert S == len(ref["table_of"])
    assert np.array_equal(tab, ref["table_of"][-1])
    assert np.array_equal(dish, np.stack(ref["dish_of"][-1]))
    assert np.array_equal(ag, ref["alpha_global"])


# ------------------------------------------ sufficient statistics
@pytest.mark.parametrize("D,path", [(32, 2), (3, 0)])
def test_parallel_stats_bitwise_vs_oracle(D, path, monkeypatch):
    """S1, S2, n of every view after warm-started sweeps (incremental updates
    at steady state, full rebuilds when more than n/8 customers move)."""
    m = _mvc()
    from mvc_amd import data
    V, K = 3, 16
    y, z = data.synthetic(4000, V, D, K, seed=40 + D)
    st = _warm_state(z, V, K)
    _path(monkeypatch, generic="1" if path == 0 else "0")
    s = m.Sampler(y, seed=13, mode="parallel")
    s.set_state(*st)
    s.sweep(6)
    assert s.zpath() & 3 == path
    ref = O.run(y, 6, 0, 1, 13, mode=O.PARALLEL, state=st)
    for v in range(V):
        g = s.stats(v)
        r = ref["stats"][v]
        assert np.array_equal(g["n"], r["n"]), v
        assert np.array_equal(g["S1"], r["S1"]), v
        assert np.array_equal(g["S2"], r["S2"]), v
    s.close()


# ---------------------------------------------------------------- sample output
def test_async_sample_output_two_chains_vs_handle():
    """mvc_run saves samples through the device snapshot ring + async D2H; with
    two chains, burn-in and thinning, every saved sample must equal the state
    read synchronously from a Sampler handle after the same sweep."""
    m = _mvc()
    from mvc_amd import data
    y, _ = data.synthetic(20000, 2, 64, 16, seed=4)
    M, burn, thin = 13, 2, 3
    res = m.run_gibbs_cpp(y, M, burn, thin, seed=17, mode="parallel", n_chains=2, quiet=True)
    saved = [it for it in range(M) if it >= burn and (it - burn) % thin == 0]
    for c in range(2):
        s = m.Sampler(y, seed=17, mode="parallel", first_chain=c)
        k = 0
        for it in range(M):
            s.sweep(1)
            if it in saved:
                t, d, h = s.state()
                assert np.array_equal(res[c]["table_of"][k], t), (c, it)
                assert np.array_equal(np.stack(res[c]["dish_of"][k]), d), (c, it)
                assert res[c]["alpha_global"][k] == h["alpha_global"]
                k += 1
        assert k == len(res[c]["table_of"])
        s.close()


def test_timing_levels_do_not_change_the_chain():
    """Coarse timing records only the whole-pass timers; switching to full
    timing at run time adds the per-phase ones.  Timing never changes the
    chain: the state equals an untimed handle's after the same sweeps."""
    m = _mvc()
    from mvc_amd import data
    y, _ = data.synthetic(20000, 2, 64, 16, seed=5)
    s = m.Sampler(y, seed=23, mode="parallel", timing="coarse")
    s.sweep(3)
    assert s.kernel_time("zresample")[1] == 3 and s.kernel_time("sweep")[1] == 3
    assert s.kernel_time("lp")[1] == 0 and s.kernel_time("hyper")[1] == 0
    s.set_timing(True)
    s.sweep(2)
    assert s.kernel_time("zresample")[1] == 5 and s.kernel_time("hyper")[1] == 2
    s.set_timing(False)
    s.sweep(1)
    assert s.kernel_time("sweep")[1] == 5
    ref = m.Sampler(y, seed=23, mode="parallel")
    ref.sweep(6)
    for a, b in zip(s.state()[:2], ref.state()[:2]):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    s.close()
    ref.close()


@pytest.mark.parametrize("waves,repair,lc", [("1", "run", "1"), ("3", "run", "1"), ("8", "grid", "1"),
                                             ("8", "run", "0"), ("3", "run", "0")])
def test_repair_shapes_same_chain(waves, repair, lc, monkeypatch):
    """The repair's execution shape does not change the chain: the run kernel
    evaluating 1, 3 or 8 customers per step (fewer waves than the V = 5
    views, so birth dish draws wrap over the waves; the lane-column
    evaluation, or lc=0 the one-wave-per-pass form), and the grid-window
    path alone (repair=grid), all bitwise vs oracle SeqSampler through the
    births of a cold start."""
    _path(monkeypatch, waves=waves, repair=repair, lc=lc)
    m = _mvc()
    from mvc_amd import data
    y, _ = data.new_simulation(1999)
    s = m.Sampler(y, seed=13, mode="parallel")
    ref = O.run(y, 10, 0, 1, seed=13, mode=O.PARALLEL)
    _check_sweeps(s, ref, 10, stats=False)
    assert sum(ref["trace_births"]) > 0
    s.close()


@pytest.mark.parametrize("waves,V", [("8", 5), ("1", 5), ("3", 3), ("8", 4)])
def test_repair_run_shapes_d16(waves, V, monkeypatch):
    """The run kernel evaluating 8, 3 or 1 customers per step (one wave each)
    gives the oracle SeqSampler chain bit for bit, through the births of a
    cold start (D = 16: S1 in the LDS cache)."""
    _path(monkeypatch, waves=waves)
    m = _mvc()
    from mvc_amd import data
    y, _ = data.synthetic(3000, V, 16, 6, seed=60 + V)
    s = m.Sampler(y, seed=17, mode="parallel")
    ref = O.run(y, 6, 0, 1, seed=17, mode=O.PARALLEL)
    _check_sweeps(s, ref, 6)
    assert sum(ref["trace_births"]) > 0 and s.repair_stats()["moves"] == ref["trace_moves"][-1]
    s.close()


_CHAINS_CHILD = r"""
import os, sys
root = sys.argv[1]
sys.path[:0] = [root, os.path.join(root, "multiview-clustering_amd")]
import numpy as np
import mvc_amd as m
from mvc_amd import data
y, _ = data.new_simulation(1999)
C, M = 4, 8
conc = m.Sampler(y, seed=21, mode="parallel", n_chains=C)          # chain-batched repair (default)
conc.sweep(M)
os.environ["MVC_PATH"] = "chain_batch=0"                          # one host thread and stream per chain
thr = m.Sampler(y, seed=21, mode="parallel", n_chains=C)
thr.sweep(M)
os.environ["MVC_PATH"] = "chain_threads=0"                        # one handle, chains one after another
ser = m.Sampler(y, seed=21, mode="parallel", n_chains=C)
ser.sweep(M)
del os.environ["MVC_PATH"]
# batched with capacity growth inside the batch (16 tables, 15 dishes at the start)
grow = m.Sampler(y, seed=21, mode="parallel", n_chains=C, table_cap=16, dish_cap=15)
for _ in range(M):
    grow.sweep(1)
assert max(grow.state(chain=c)[1].shape[1] for c in range(C)) > 16
for c in range(C):
    one = m.Sampler(y, seed=21, mode="parallel", first_chain=c)
    one.sweep(M)
    t1, d1, h1 = one.state()
    for s in (conc, thr, ser, grow):
        t, d, h = s.state(chain=c)
        assert np.array_equal(t, t1) and np.array_equal(d, d1), c
        assert h["sigma_global"] == h1["sigma_global"] and np.array_equal(h["tau_v"], h1["tau_v"])
    one.close()
for s in (conc, thr, ser, grow):
    s.close()
print("chains OK")
"""


def test_chains_concurrent_equal_serial():
    """Several chains in one handle (ChainSet, shared device data): the
    chain-batched repair (one launch per round for all chains), the per-chain
    streams and host threads (MVC_PATH chain_batch=0) and the serial loop
    (chain_threads=0) all equal the same chain run alone (first_chain =
    c), bit for bit, through a cold start with births, also when the batch
    grows the chains' capacities."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _CHAINS_CHILD, root], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "chains OK" in r.stdout, (r.stdout[-1000:], r.stderr[-2000:])


@pytest.mark.parametrize("env", [
    {"lc": "0"},                                      # batched kind 0: one wave per customer, LDS cache
    {"lc": "col"},                                    # batched kind 3: lane columns (no lane loop)
    {},                                               # batched kind 6: the small chains' lane loop (lane_batch)
    {"run_lds": "0", "wide": "0"},                    # kind 0 on the global layout
    {"run_lds": "0", "wide": "block"},                # kind 2: the block-wide evaluation
    {"run_lds": "0"},                                 # grid-wide evaluation: every chain on its own stream
    {"repair": "grid"},                               # grid windows only: every chain on its own stream
], ids=["lc0", "lane_columns", "lane8", "global_tw1", "wide_block", "wide_grid", "grid_only"])
def test_chains_batched_kinds_equal_alone(env, monkeypatch):
    """The chain-batched repair with every run-kernel instance it can batch
    (kinds 0 and 2) and with the chains it launches one by one on their own
    streams (grid-wide evaluation, grid-only repair: their window evaluation
    must not also run in the batched window launch) gives every chain bit for
    bit as the same chain swept alone, through a cold start with births."""
    _path(monkeypatch, **env)
    m = _mvc()
    from mvc_amd import data
    y, _ = data.new_simulation(1999)
    C, M = 3, 6
    conc = m.Sampler(y, seed=31, mode="parallel", n_chains=C)
    conc.sweep(M)
    for c in range(C):
        one = m.Sampler(y, seed=31, mode="parallel", first_chain=c)
        one.sweep(M)
        t1, d1, h1 = one.state()
        t, d, h = conc.state(chain=c)
        assert np.array_equal(t, t1) and np.array_equal(d, d1), c
        assert h["sigma_global"] == h1["sigma_global"] and np.array_equal(h["tau_v"], h1["tau_v"]), c
        one.close()
    ref = O.run(y, M, 0, 1, seed=31, chain=1, mode=O.PARALLEL)
    assert np.array_equal(conc.state(chain=1)[0], ref["table_of"][-1])
    conc.close()


def test_lane_batch_transitions_equal_alone():
    """ChainSet's lane_batch sweeps (every chain in the lane loop: the repair's
    init, compaction, MH and status read-back batched over the chains on one
    stream) and its other sweeps alternate through the reference call's cold
    start (the tables outgrow the lane loop, then shrink back into it); every
    chain stays bit for bit the chain swept alone, sweep by sweep, and
    mvc_run's samples (save_all_async after lane_batch sweeps, the chains' own
    saves after the others) equal the one-chain calls'."""
    m = _mvc()
    from mvc_amd import data
    y, _ = data.new_simulation(7)
    C, M = 4, 24
    conc = m.Sampler(y, seed=13, mode="parallel", n_chains=C)
    alone = [m.Sampler(y, seed=13, mode="parallel", first_chain=c) for c in range(C)]
    lane, other = 0, 0
    for it in range(M):
        conc.sweep(1)
        if conc.zpath() & 256:
            lane += 1
        else:
            other += 1
        for c in range(C):
            alone[c].sweep(1)
            t1, d1, h1 = alone[c].state()
            t, d, h = conc.state(chain=c)
            assert np.array_equal(t, t1) and np.array_equal(d, d1), (it, c)
            assert np.array_equal(h["tau_v"], h1["tau_v"]) and h["alpha_global"] == h1["alpha_global"], (it, c)
    assert lane > 0 and other > 0, (lane, other)
    conc.close()
    for a in alone:
        a.close()
    multi = m.run_gibbs_cpp(y, M, M // 3, 1, seed=13, mode="parallel", n_chains=C, quiet=True)
    for c, res in enumerate(multi):
        _compare(res, m.run_gibbs_cpp(y, M, M // 3, 1, seed=13, mode="parallel", first_chain=c, quiet=True))


_LAST_BIRTH_CHILD = r"""
import os, sys
root = sys.argv[1]
sys.path[:0] = [root, os.path.join(root, "multiview-clustering_amd")]
import numpy as np
import mvc_amd as m
from mvc_amd import data
from oracle import oracle as O
y, _ = data.new_simulation(1)
n, C, M = y.shape[1], 4, 12
res = m.run_gibbs_cpp(y, M, 0, 1, seed=1, mode="parallel", n_chains=C, quiet=True)
last = 0
for c in range(C):
    ref = O.run(y, M, 0, 1, 1, chain=c, mode=O.PARALLEL)
    for s in range(M):
        assert np.array_equal(res[c]["table_of"][s], ref["table_of"][s]), (c, s)
        assert np.array_equal(np.stack(res[c]["dish_of"][s]), ref["dish_of"][s]), (c, s)
        t = ref["table_of"][s]
        last += int(np.bincount(t)[t[n - 1]] == 1)   # the last customer sits alone: a birth
    assert np.array_equal(res[c]["sigma_global"], ref["sigma_global"]), c
print("last-birth OK", last)
"""


@pytest.mark.parametrize("vp", ["0", "1", "col"])
def test_last_customer_birth_with_poisoned_lds(vp):
    """Regression test of the round-3 multi-chain fault: a
    birth decided for the sweep's LAST customer is committed by the birth
    kernel, and the next repair round's run kernel then starts at cur == n.
    The New_Simulation shape with seed 1 has such births in every chain
    (19 over 4 chains x 12 cold sweeps; the oracle counts them below, since
    only a birth can leave the last customer alone at a table).  Four
    chains run concurrently in one handle with the run kernel's LDS filled
    with 0xA5 at every launch (MVC_LDS_FILL: a read of a ring slot the
    launch never wrote sees the same garbage every time) and every index a
    run-kernel commit writes through checked (MVC_RUN_CHECK: a bad one fails
    the sweep with the check's number instead of storing).  Without the fix
    the value-prediction loop read pcs[depth - 1] and ring slots at cur == n
    and the check fired (round 4: check 10, i0 = n); with it every chain is
    bitwise the oracle's."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # vp = "1": value prediction at N = 200 too (small chains run the lane
    # loop by default, MVC_PATH small_plain), the loop the fault was in; "col":
    # the plain lane-column loop; "0": the small chains' default (lane loop)
    path = {"1": "small_plain=0", "col": "lc=col", "0": ""}[vp]
    env = dict(os.environ, MVC_LDS_FILL="0xA5", MVC_RUN_CHECK="1", MVC_PATH=path)
    r = subprocess.run([sys.executable, "-c", _LAST_BIRTH_CHILD, root], capture_output=True, text=True, timeout=240,
                       env=env)
    assert r.returncode == 0 and "last-birth OK" in r.stdout, (r.stdout[-1000:], r.stderr[-2000:])
    assert int(r.stdout.split("last-birth OK")[1].split()[0]) >= 4


@pytest.mark.parametrize("force", ["", "1", "d256", "d256-runtime", "d256-separate"])
def test_dish_block_producer(force, monkeypatch):
    """The dish-block MFMA producer (mvc_par_lpbig_kernel: A-fragments from y
    itself, dishes in blocks of 64, the view maximum combined over blocks):
    K_v = 128 / 64 / 32 at D = 32 (two dish blocks in view 0, the runtime
    k-step loop), warm; forced onto a K <= 64 shape that the tiled producer
    would take (D = 64: the unrolled tile); and configs[4]'s D = 256 with
    K_v = 80 / 40 (a 64 + 16 dish split), unrolled and with the runtime loop
    (MVC_PATH big_sp=runtime).  A view with two or more dish blocks runs them
    in one XCD-grouped launch (mvc_par_lpbig_group_kernel, the view maximum
    an atomic max) unless MVC_PATH big_group=0 ("d256-separate": one launch
    per block, the maximum combined in block order); bitwise vs the oracle."""
    if force:
        _path(monkeypatch, big="1", **({"big_sp": "runtime"} if force == "d256-runtime" else
                                       {"big_group": "0"} if force == "d256-separate" else {}))
    m = _mvc()
    from mvc_amd import data
    N, V, D, K = {"": (6000, 3, 32, 128), "1": (4100, 4, 64, 64)}.get(force, (3000, 2, 256, 80))
    y, z = data.synthetic(N, V, D, K, seed=17)
    st = _warm_state(z, V, K)
    s = m.Sampler(y, seed=5, mode="parallel")
    s.set_state(*st)
    ref = O.run(y, 3, 0, 1, seed=5, mode=O.PARALLEL, state=st)
    _check_sweeps(s, ref, 3)
    assert s.zpath() & 64   # the dish-block producer ran
    s.close()


@pytest.mark.parametrize("world", [2, 3])
def test_shard_ranks_equal_unsharded(world, tmp_path):
    """Within-chain N-sharding (mvc_sampler_set_shard): `world` processes on
    one GPU each evaluate phase A for their shard, all-gather the choices
    (gloo through host memory) and run the same repair; every rank's chain
    equals the unsharded chain bit for bit, through a cold start (movers
    in every sweep, the last shard ragged)."""
    import socket
    import subprocess
    import sys
    N, V, D, K, sweeps = 20000 + 37, 3, 16, 8, 4
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    here = os.path.dirname(os.path.abspath(__file__))
    procs = [subprocess.Popen([sys.executable, os.path.join(here, "shard_worker.py"), str(r), str(world), str(port),
                               str(tmp_path / f"r{r}.npz"), str(N), str(V), str(D), str(K), str(sweeps)])
             for r in range(world)]
    rcs = [p.wait(timeout=150) for p in procs]
    assert rcs == [0] * world, rcs
    m = _mvc()
    from mvc_amd import data
    y, _ = data.synthetic(N, V, D, K, seed=31)
    s = m.Sampler(y, seed=5, mode="parallel")
    for it in range(sweeps):
        s.sweep(1)
        t, d, h = s.state()
        for r in range(world):
            z = np.load(tmp_path / f"r{r}.npz")
            assert np.array_equal(z["t"][it], t), (r, it)
            assert np.array_equal(z["tau"][it], h["tau_v"]), (r, it)
            if it == sweeps - 1:
                assert np.array_equal(z["d"], d) and int(z["moves"]) == s.repair_stats()["moves"], r
                assert int(z["calls"]) == sweeps, r   # one exchange per sweep
    assert s.repair_stats()["moves"] > 0
    s.close()


@pytest.mark.parametrize("wide,V,fin", [("1", 3, "1"), ("1", 3, "0"), ("0", 3, "1"), ("1", 5, "1"), ("1", 5, "0"),
                                        ("block", 3, "1"), ("block", 5, "1")])
def test_repair_global_wide(wide, V, fin, monkeypatch):
    """The run kernel on its global-scratch layout (MVC_PATH run_lds=0, as
    when the state outgrows the LDS): one customer over the grid (wide=1: lp
    kernel + fin kernel, the fin kernel's evaluation in LDS or, wide_fin=0,
    in the global scratch), over the whole block (seq_resample_wide: dishes,
    tables and scans split over the 8 waves) or one customer per wave
    (wide=0); bitwise vs oracle SeqSampler through the births of a cold
    start."""
    _path(monkeypatch, run_lds="0", wide=wide, wide_fin=fin)
    m = _mvc()
    from mvc_amd import data
    y, _ = data.synthetic(3000, V, 16, 6, seed=80 + V)
    s = m.Sampler(y, seed=19, mode="parallel")
    ref = O.run(y, 5, 0, 1, seed=19, mode=O.PARALLEL)
    _check_sweeps(s, ref, 5)
    assert sum(ref["trace_births"]) > 0 and s.repair_stats()["moves"] == ref["trace_moves"][-1]
    s.close()


@pytest.mark.parametrize("mode", ["parallel", "exact"])
def test_run_chain_ids_and_pooled_summary(mode):
    """mvc_run's chain ids (first_chain + c * chain_stride: the layout the
    multi-device split uses, chain c of n_devices on device c % n_devices)
    give every chain the chain a one-chain call with that id gives, bit for
    bit; mvc_result_summary's pooled means and R-hat equal a host
    computation over the saved draws."""
    m = _mvc()
    from mvc_amd import data
    from mvc_amd import _lib as L
    from mvc_amd.sampler import make_config, _view_ptrs, _views_to_array
    import ctypes
    y, _ = data.new_simulation(3)
    M, burn = 30, 10
    V = y.shape[0]
    summ = {}
    multi = m.run_gibbs_cpp(y, M, burn, 1, seed=99, mode=mode, n_chains=3, n_devices=1, summary=summ)
    for c, res in enumerate(multi):
        one = m.run_gibbs_cpp(y, M, burn, 1, seed=99, mode=mode, first_chain=c)
        _compare(res, one)
    # chain_stride: ids 1, 3, 5
    yy = _views_to_array(y)
    cfg = make_config(yy.shape[1], V, 1, M, burn, 1, 99, 3, 1, 0, mode, n_devices=1, chain_stride=2)
    lib = L.lib()
    r = ctypes.c_void_p()
    buf = L.errbuf()
    L.check(lib.mvc_run(ctypes.byref(cfg), _view_ptrs(yy), ctypes.byref(r), buf, len(buf)), buf)
    try:
        for c, gid in enumerate((1, 3, 5)):
            one = m.run_gibbs_cpp(y, M, burn, 1, seed=99, mode=mode, first_chain=gid)
            t = np.ctypeslib.as_array(lib.mvc_result_table_of(r, c, M - burn - 1), shape=(yy.shape[1],))
            assert np.array_equal(t, one["table_of"][-1]), gid
    finally:
        lib.mvc_result_free(r)
    H = np.stack([np.concatenate([np.stack(res["tau_v"]).T, np.stack(res["alpha_v"]).T, np.stack(res["sigma_v"]).T,
                                  res["alpha_global"][:, None], res["sigma_global"][:, None]], axis=1)
                  for res in multi])                                       # [C][S][3V+2]
    assert np.allclose(summ["mean"], H.mean(axis=(0, 1)), rtol=1e-12, atol=0)
    C, S = H.shape[0], H.shape[1]
    cm, cv = H.mean(1), H.var(1, ddof=1)
    B = S * cm.var(0, ddof=1)
    W = cv.mean(0)
    with np.errstate(divide="ignore", invalid="ignore"):
        rh = np.sqrt(((S - 1) / S * W + B / S) / W)
    assert np.allclose(summ["rhat"], rh, rtol=1e-10, equal_nan=True)


@pytest.mark.parametrize("mode", ["exact", "parallel"])
def test_run_n_devices_split(mode):
    """mvc_run with n_devices = 2 (one host thread per device, chain c on
    device c % 2 with global id first_chain + c): every chain equals a
    one-chain call with that id, bit for bit, and the pooled summary covers
    all chains.  Needs two visible GPUs (skipped on the one-GPU boxes)."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs")
    m = _mvc()
    from mvc_amd import data
    y, _ = data.new_simulation(5)
    M, burn = 20, 10
    summ = {}
    multi = m.run_gibbs_cpp(y, M, burn, 1, seed=7, mode=mode, n_chains=4, n_devices=2, summary=summ)
    assert len(multi) == 4
    for c, res in enumerate(multi):
        one = m.run_gibbs_cpp(y, M, burn, 1, seed=7, mode=mode, first_chain=c)
        _compare(res, one)
    assert summ["mean"].shape == (3 * y.shape[0] + 2,)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["exact", "parallel"])
def test_run_n_devices_split_on_one_gpu(mode, monkeypatch):
    """The same n_devices = 2 split with both logical devices mapped to
    device 0 (MVC_DEVICE_MAP=0,0): mvc_run's per-device host threads, the
    chain striding (device d holds chains d, d + 2, ... with ids first_chain
    + c) and the result interleave run on one MI355X.  Every chain equals a
    one-chain call with its id, bit for bit, and the pooled summary equals
    the one of the same chains run on one logical device."""
    m = _mvc()
    from mvc_amd import data
    y, _ = data.new_simulation(5)
    M, burn = 20, 10
    s1, s2 = {}, {}
    single = m.run_gibbs_cpp(y, M, burn, 1, seed=7, mode=mode, n_chains=5, summary=s1)
    monkeypatch.setenv("MVC_DEVICE_MAP", "0,0")
    multi = m.run_gibbs_cpp(y, M, burn, 1, seed=7, mode=mode, n_chains=5, n_devices=2, summary=s2)
    assert len(multi) == 5
    for c, res in enumerate(multi):
        _compare(res, single[c])
        if c in (0, 3):
            _compare(res, m.run_gibbs_cpp(y, M, burn, 1, seed=7, mode=mode, first_chain=c))
    assert np.array_equal(s1["mean"], s2["mean"])
    assert np.array_equal(s1["rhat"], s2["rhat"], equal_nan=True)
    monkeypatch.setenv("MVC_DEVICE_MAP", "0,9")
    with pytest.raises(Exception, match="MVC_DEVICE_MAP"):
        m.run_gibbs_cpp(y, 2, 0, 1, seed=7, mode=mode, n_chains=2, n_devices=2)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["exact", "parallel"])
def test_run_eight_logical_devices_on_one_gpu(mode, monkeypatch):
    """mvc_run's 8-way split (the driver's 8-GPU node shape) on one MI355X:
    n_devices = 8 with every logical device mapped to device 0
    (MVC_DEVICE_MAP=0,...,0), 16 chains striped two per device.  Every chain
    equals the same chain run on one logical device, bit for bit, and so
    does the pooled summary."""
    m = _mvc()
    from mvc_amd import data
    y, _ = data.new_simulation(11)
    M, burn, C = 12, 6, 16
    s1, s8 = {}, {}
    single = m.run_gibbs_cpp(y, M, burn, 1, seed=9, mode=mode, n_chains=C, summary=s1)
    monkeypatch.setenv("MVC_DEVICE_MAP", ",".join(["0"] * 8))
    multi = m.run_gibbs_cpp(y, M, burn, 1, seed=9, mode=mode, n_chains=C, n_devices=8, summary=s8)
    assert len(multi) == C
    for c in range(C):
        _compare(multi[c], single[c])
    assert np.array_equal(s1["mean"], s8["mean"])
    assert np.array_equal(s1["rhat"], s8["rhat"], equal_nan=True)


def test_shard_exchange_failure_leaves_the_chain_unchanged():
    """A failing all_gather (the callback returns nonzero) stops the sweep
    with MVC_ERR_CALLBACK before the exchange buffer is read: the state is
    the state before the sweep, and the handle sweeps on normally after a
    working exchange is installed."""
    m = _mvc()
    from mvc_amd import data
    import torch

    from mvc_amd.dist import shard_len

    class Failing:
        def __init__(self, n):
            self.buf = torch.zeros(2 * shard_len(n, 2), dtype=torch.int32, device="cuda")
            self.ptr = self.buf.data_ptr()

        def all_gather(self):
            raise RuntimeError("exchange down")

    y, _ = data.synthetic(4000, 2, 16, 6, seed=3)
    s = m.Sampler(y, seed=5, mode="parallel")
    s.sweep(1)
    before = s.state()
    s.set_shard(0, 2, Failing(4000))
    with pytest.raises(RuntimeError, match="shard exchange failed"):
        s.sweep(1)
    after = s.state()
    assert np.array_equal(before[0], after[0]) and np.array_equal(before[1], after[1])
    assert before[2]["sigma_global"] == after[2]["sigma_global"]
    assert s.sweeps_done == 1
    s.set_shard(0, 1)
    s.sweep(1)
    ref = m.Sampler(y, seed=5, mode="parallel")
    ref.sweep(2)
    assert np.array_equal(s.state()[0], ref.state()[0])
    s.close()
    ref.close()


def test_table_limit_is_a_clean_error(monkeypatch):
    """A cold start that needs more tables than the parallel mode's limit
    (262,144 = 64^3, the MH's three-level tree64; lowered here with
    MVC_PATH max_tables) fails with MVC_ERR_UNSUPPORTED and a message naming the
    limit, not a wrong answer (configs[3] at N = 1M from the
    reference initialisation would reach it: nearly every customer opens a
    table in sweep 0, multiview_gibbs.cpp:94)."""
    _path(monkeypatch, max_tables="32")
    m = _mvc()
    from mvc_amd import data
    y, _ = data.new_simulation(1999)          # opens ~70 tables in sweep 0
    s = m.Sampler(y, seed=5, mode="parallel", table_cap=16)
    with pytest.raises(m.MvcError, match="limit 32 tables") as e:
        s.sweep(3)
    assert e.value.code == 4                  # MVC_ERR_UNSUPPORTED
    s.close()


@pytest.mark.parametrize("V,D,K,vp", [(4, 1, 16, "1"), (4, 1, 16, "0"), (2, 16, 8, "1"), (5, 4, 12, "1")])
def test_value_prediction_same_chain(V, D, K, vp, monkeypatch, capfd):
    """Value prediction (the lane-column run kernel evaluating customers i ..
    i+3 against the state with the phase-A choices of the ones before applied,
    mvc_repair.h seq_run_loop_vp) gives the oracle SeqSampler chain bit for
    bit from a warm state where most customers move (overlapping clusters) and
    through births; MVC_PATH vp=0 is the plain lane-column loop on the same chain."""
    _path(monkeypatch, vp=vp, vp_stats="1")
    m = _mvc()
    import bench
    from mvc_amd import data
    y, z = data.synthetic(20_000, V, D, K, seed=70 + V + D, sd=1.3 if D == 1 else 4.0)
    st = bench.warm_state(z, V, K)
    s = m.Sampler(y, seed=21, mode="parallel")
    s.set_state(*st)
    ref = O.run(y, 3, 0, 1, seed=21, mode=O.PARALLEL, state=st)
    for it in range(3):
        s.sweep(1)
        t, d, h = s.state()
        assert np.array_equal(t, ref["table_of"][it]), it
        assert np.array_equal(d, ref["dish_of"][it]), it
        assert np.array_equal(h["tau_v"], ref["tau_v"][:, it]), it
    rep = s.repair_stats()
    s.close()
    err = capfd.readouterr().err
    steps = sum(int(l.split()[3]) for l in err.splitlines() if l.startswith("mvc vp steps"))
    assert rep["moves"] > 0
    if vp == "1":
        assert steps > 0, "value prediction did not run"
    else:
        assert steps == 0


# ------------------------------------------------ several sweeps per call
@pytest.mark.parametrize("cap", [(256, 128), (8, 4)])
def test_exact_sweeps_per_launch(cap):
    """Several sweeps in one kernel launch (Sampler.sweep(k)) equal k calls
    of one sweep, with and without capacity growth inside the launch."""
    m = _mvc()
    from mvc_amd import data
    y, _ = data.config1(1, n=600)
    a = m.Sampler(y, seed=7, mode="exact", n_chains=3, table_cap=cap[0], dish_cap=cap[1])
    b = m.Sampler(y, seed=7, mode="exact", n_chains=3, table_cap=cap[0], dish_cap=cap[1])
    for k in (1, 2, 5, 11):
        a.sweep(k)
        for _ in range(k):
            b.sweep(1)
        for c in range(3):
            ta, da, ha = a.state(c)
            tb, db, hb = b.state(c)
            assert np.array_equal(ta, tb), (k, c)
            assert np.array_equal(da, db), (k, c)
            assert ha["alpha_global"] == hb["alpha_global"], (k, c)
    a.close()
    b.close()


@pytest.mark.parametrize("warm", [False, True])
def test_parallel_sweeps_per_call(warm):
    """Sampler.sweep(k) equals k calls of sweep(1): a cold start (moves,
    births, capacity growth) and a warm start, and the warm chain equals the
    oracle."""
    m = _mvc()
    from mvc_amd import data
    y, z = data.synthetic(5000, 4, 128, 64, seed=77)
    st = None
    if warm:
        uniq, table_of = np.unique(z, return_inverse=True)
        T = uniq.size
        dish = np.stack([np.arange(T) % max(1, 64 // (2 ** v)) for v in range(4)]).astype(np.int32)
        st = (table_of.astype(np.int32), dish, np.array([1.69] * 4 + [1.0] * 4 + [0.5] * 4 + [1.0, 0.6]))
    caps = {} if warm else dict(table_cap=16, dish_cap=8)   # cold: growth inside sweep(k)
    a = m.Sampler(y, seed=21, mode="parallel", **caps)
    b = m.Sampler(y, seed=21, mode="parallel", **caps)
    if st is not None:
        a.set_state(*st)
        b.set_state(*st)
    for k in (1, 3, 4):
        a.sweep(k)
        for _ in range(k):
            b.sweep(1)
        ta, da, ha = a.state()
        tb, db, hb = b.state()
        assert np.array_equal(ta, tb), k
        assert np.array_equal(da, db), k
        assert ha["sigma_global"] == hb["sigma_global"], k
    if warm:
        ref = O.run(y, 8, 0, 1, seed=21, mode=O.PARALLEL, state=st)
        t, d, h = a.state()
        assert np.array_equal(t, ref["table_of"][7])
        assert np.array_equal(d, ref["dish_of"][7])
    a.close()
    b.close()
