"""ctypes binding of the CPU oracle (oracle/build/libmvc_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product never imports this module.

Parity status: "parity unpinned" against the reference binary (the reference
needs Rcpp/R, absent here; see mvc_oracle.cpp header and DESIGN.md §3).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libmvc_oracle.so")
_lib = None

# EXACT: the reference schedule, literal (D = 1).  PARALLEL: the same
# sequential schedule with the GPU-shaped conditional and counter-addressed
# Philox draws -- the spec libmvc_hip.so's parallel mode executes (DESIGN.md
# §4.8).  JACOBI: every customer against the sweep-start state (round 1's
# schedule; kept only to document that it does NOT sample the reference's
# posterior, tests/test_posterior.py).
EXACT, PARALLEL, JACOBI = 0, 1, 3
LIBM, PORTABLE = 0, 1


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i32, u64, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_int64
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int)
        L.mvo_run.restype = vp
        L.mvo_run.argtypes = [dp, i32, i32, i32, i32, i32, i32, u64, i32, i32, i32]
        L.mvo_run_from.restype = vp
        L.mvo_run_from.argtypes = [dp, i32, i32, i32, i32, i32, i32, u64, i32, i32, i32, ip, i32, ip, dp]
        L.mvo_error.restype = ctypes.c_char_p
        L.mvo_error.argtypes = [vp]
        for f in ("mvo_num_saved", "mvo_num_sweeps"):
            getattr(L, f).restype = i32
            getattr(L, f).argtypes = [vp]
        L.mvo_sample_T.restype = i32
        L.mvo_sample_T.argtypes = [vp, i32]
        L.mvo_copy_table_of.argtypes = [vp, i32, ip]
        L.mvo_copy_dish_of.argtypes = [vp, i32, ip]
        L.mvo_copy_hyper.argtypes = [vp, dp, dp, dp, dp, dp]
        L.mvo_copy_trace.argtypes = [vp, ip, ctypes.POINTER(ctypes.c_uint64)]
        L.mvo_copy_trace_moves.argtypes = [vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                           ctypes.POINTER(ctypes.c_int64)]
        L.mvo_copy_trace_underflow.argtypes = [vp] + [ctypes.POINTER(ctypes.c_int64)] * 4
        L.mvo_free.argtypes = [vp]
        L.mvo_stats_K.restype = i32
        L.mvo_stats_K.argtypes = [vp, i32]
        L.mvo_copy_stats.argtypes = [vp, i32, dp, dp, ip]
        for f in ("mvo_pm_exp", "mvo_pm_log", "mvo_pm_lgamma", "mvo_pm_qnorm"):
            getattr(L, f).argtypes = [dp, dp, i64]
        L.mvo_philox.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.POINTER(ctypes.c_uint32)]
        L.mvo_seq_uniforms.argtypes = [u64, ctypes.c_uint32, u64, dp, i64]
        L.mvo_tree64_sum.restype = ctypes.c_double
        L.mvo_tree64_sum.argtypes = [dp, i64]
        L.mvo_phase_a.restype = i32
        L.mvo_phase_a.argtypes = [i32, i32, i32, ip, i32, ip, dp, ip, dp, dp, ip, u64, i32, i32, i32, ip, dp, ip,
                                  ctypes.c_char_p, i32]
        L.mvo_tree64_select.restype = i64
        L.mvo_tree64_select.argtypes = [dp, i64, ctypes.c_double]
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def run(y, M, burn_in, thin, seed, chain=0, mode=EXACT, math=PORTABLE, state=None):
    """Run one chain.  y: float64 array [V][n] (D=1) or [V][n][D].

    state = (table_of[n], dish_of[V][T], hyper[3V+2]) starts the chain from
    that state (mirror of mvc_sampler_set_state) instead of the reference
    initialisation.

    Returns a dict shaped like the reference's Rcpp::List
    (multiview_gibbs.cpp:121-130) plus per-sweep traces.
    """
    y = np.ascontiguousarray(y, dtype=np.float64)
    if y.ndim == 2:
        y = y[:, :, None]
    V, n, D = y.shape
    L = lib()
    if state is None:
        h = L.mvo_run(_dp(y), n, V, D, M, burn_in, thin, ctypes.c_uint64(seed), chain, mode, math)
    else:
        tab = np.ascontiguousarray(state[0], dtype=np.int32)
        dsh = np.ascontiguousarray(state[1], dtype=np.int32)
        hyp = np.ascontiguousarray(state[2], dtype=np.float64)
        ipt = ctypes.POINTER(ctypes.c_int)
        h = L.mvo_run_from(_dp(y), n, V, D, M, burn_in, thin, ctypes.c_uint64(seed), chain, mode, math,
                           tab.ctypes.data_as(ipt), dsh.shape[1], dsh.ctypes.data_as(ipt), _dp(hyp))
    try:
        err = L.mvo_error(h)
        if err:
            raise RuntimeError(err.decode())
        S = L.mvo_num_saved(h)
        table_of, dish_of = [], []
        for s in range(S):
            t = np.empty(n, dtype=np.int32)
            L.mvo_copy_table_of(h, s, t.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
            T = L.mvo_sample_T(h, s)
            dd = np.empty(V * T, dtype=np.int32)
            L.mvo_copy_dish_of(h, s, dd.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
            table_of.append(t)
            dish_of.append(dd.reshape(V, T))
        av, sv, tv = (np.empty(S * V) for _ in range(3))
        ag, sg = np.empty(S), np.empty(S)
        L.mvo_copy_hyper(h, _dp(av), _dp(sv), _dp(tv), _dp(ag), _dp(sg))
        stats = []
        for v in range(V):
            K = L.mvo_stats_K(h, v)
            if K:
                s1, s2, nk = np.empty((K, D)), np.empty(K), np.empty(K, dtype=np.int32)
                L.mvo_copy_stats(h, v, _dp(s1), _dp(s2), nk.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
                stats.append({"S1": s1, "S2": s2, "n": nk})
        nsw = L.mvo_num_sweeps(h)
        tT = np.empty(nsw, dtype=np.int32)
        td = np.empty(nsw, dtype=np.uint64)
        L.mvo_copy_trace(h, tT.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                         td.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
        tm, tb, tn = (np.empty(nsw, dtype=np.int64) for _ in range(3))
        i64p = ctypes.POINTER(ctypes.c_int64)
        L.mvo_copy_trace_moves(h, tm.ctypes.data_as(i64p), tb.ctypes.data_as(i64p), tn.ctypes.data_as(i64p))
        uf = [np.empty(nsw, dtype=np.int64) for _ in range(4)]
        L.mvo_copy_trace_underflow(h, *(a.ctypes.data_as(i64p) for a in uf))
        return {
            "table_of": table_of,
            "dish_of": dish_of,
            "alpha_v": av.reshape(S, V).T.copy(),
            "sigma_v": sv.reshape(S, V).T.copy(),
            "tau_v": tv.reshape(S, V).T.copy(),
            "alpha_global": ag,
            "sigma_global": sg,
            "trace_T": tT,
            "trace_draws": td,
            "trace_moves": tm,         # PARALLEL mode: customers that changed table, per sweep (else -1)
            "trace_births": tb,
            "trace_newdish": tn,
            # EXACT mode, per sweep: the reference's linear-space underflow
            # (table-0 fallbacks, underflowed tables summed over customers,
            # customers with one, underflowed new-table probabilities)
            "trace_fallback": uf[0], "trace_uf_tables": uf[1], "trace_uf_customers": uf[2], "trace_uf_new": uf[3],
            "stats": stats,            # parallel mode: final S1 [K][D], S2, n per view
        }
    finally:
        L.mvo_free(h)


def phase_a(table_of, dish_of, hyper, stats, seed, chain, sweep, idx, rows):
    """Phase-A draws (the sweep-start conditional, ParallelSampler::
    resample_customer) of customers idx given the state as a partition
    (table_of[n], dish_of[V][T] raw ids, hyper[3V+2]) plus per-view stats
    (list of dicts S1 [K][D], S2 [K], n [K] in ascending raw id, as
    Sampler.stats returns them) and only those customers' rows
    rows[m][V][D].  For checks at sizes where y is not on the host."""
    tab = np.ascontiguousarray(table_of, dtype=np.int32)
    dsh = np.ascontiguousarray(dish_of, dtype=np.int32)
    hyp = np.ascontiguousarray(hyper, dtype=np.float64)
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    rows = np.ascontiguousarray(rows, dtype=np.float64)
    m, V, D = rows.shape
    K = np.array([st["n"].size for st in stats], dtype=np.int32)
    S1 = np.ascontiguousarray(np.concatenate([np.asarray(st["S1"], dtype=np.float64).ravel() for st in stats]))
    S2 = np.ascontiguousarray(np.concatenate([np.asarray(st["S2"], dtype=np.float64) for st in stats]))
    nk = np.ascontiguousarray(np.concatenate([np.asarray(st["n"], dtype=np.int32) for st in stats]))
    out = np.empty(m, dtype=np.int32)
    err = ctypes.create_string_buffer(512)
    ipt = ctypes.POINTER(ctypes.c_int)
    rc = lib().mvo_phase_a(tab.size, V, D, tab.ctypes.data_as(ipt), dsh.shape[1], dsh.ctypes.data_as(ipt), _dp(hyp),
                           K.ctypes.data_as(ipt), _dp(S1), _dp(S2), nk.ctypes.data_as(ipt), ctypes.c_uint64(seed),
                           chain, sweep, m, idx.ctypes.data_as(ipt), _dp(rows), out.ctypes.data_as(ipt), err, 512)
    if rc != 0:
        raise RuntimeError(err.value.decode())
    return out


def _vec(fn, x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    o = np.empty_like(x)
    fn(_dp(x), _dp(o), x.size)
    return o


def pm_exp(x):
    return _vec(lib().mvo_pm_exp, x)


def pm_log(x):
    return _vec(lib().mvo_pm_log, x)


def pm_lgamma(x):
    return _vec(lib().mvo_pm_lgamma, x)


def pm_qnorm(x):
    return _vec(lib().mvo_pm_qnorm, x)


def philox(ctr, key):
    c = (ctypes.c_uint32 * 4)(*ctr)
    o = (ctypes.c_uint32 * 4)()
    lib().mvo_philox(c, ctypes.c_uint32(key[0]), ctypes.c_uint32(key[1]), o)
    return tuple(o)


def seq_uniforms(seed, chain, start, n):
    o = np.empty(n)
    lib().mvo_seq_uniforms(ctypes.c_uint64(seed), chain, ctypes.c_uint64(start), _dp(o), n)
    return o


def tree64_sum(x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    return lib().mvo_tree64_sum(_dp(x), x.size)


def tree64_select(x, r):
    x = np.ascontiguousarray(x, dtype=np.float64)
    return int(lib().mvo_tree64_select(_dp(x), x.size, r))


def ari(a, b):
    """Adjusted Rand index, restating mcclust::arandi(cl1, cl2, adjust = TRUE)
    (the ARI of New_Simulation.R:5,189; mcclust is an R package absent here,
    restated from its published source):
        tab.1 <- table(cl1); tab.2 <- table(cl2); tab.12 <- table(cl1, cl2)
        correc <- sum(choose(tab.1,2)) * sum(choose(tab.2,2)) / choose(n,2)
        (sum(choose(tab.12,2)) - correc) /
            (0.5*sum(choose(tab.1,2)) + 0.5*sum(choose(tab.2,2)) - correc)
    R's choose(k, 2) of a count is the exact integer (nmath choose.c), so the
    three pair sums are exact integers; the fp64 expression then runs in R's
    left-to-right order.  A 1 x 1 table is 0/0 = NaN, as in R.  Pinned
    against scikit-learn's adjusted_rand_score (the same Hubert-Arabie index)
    in tests/test_ari.py."""
    a = np.asarray(a).ravel().astype(np.int64)
    b = np.asarray(b).ravel().astype(np.int64)
    assert a.shape == b.shape
    n = int(a.size)

    def pair_sum(labels):   # sum(choose(table(labels), 2)), exact integer
        _, cnt = np.unique(labels, return_counts=True, axis=0)
        cnt = cnt.astype(np.int64)
        return int(np.sum(cnt * (cnt - 1) // 2))

    A = pair_sum(np.stack([a, b], axis=1))
    SA, SB = pair_sum(a), pair_sum(b)
    a_, sa, sb = np.float64(A), np.float64(SA), np.float64(SB)
    nn = np.float64(n * (n - 1) // 2)
    with np.errstate(divide="ignore", invalid="ignore"):
        correc = (sa * sb) / nn
        return float((a_ - correc) / ((np.float64(0.5) * sa + np.float64(0.5) * sb) - correc))
