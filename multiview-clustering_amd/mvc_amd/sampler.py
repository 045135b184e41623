"""Python host mirror of the reference's R entry point.

``run_gibbs_cpp(data_views, M, burn_in, thin)`` has the argument meaning and
the output list of ``Rcpp::List run_gibbs_cpp(const Rcpp::List& data_views,
int M, int burn_in, int thin)`` (/root/reference/Multiview/multiview_gibbs.cpp:
105-131): a dict with ``table_of`` (list over saved iterations of int32[n],
0-based table positions), ``dish_of`` (list over saved iterations of a list
over views of int32[T_s], raw dish ids) -- both read-only sequences whose
items are built on access from one contiguous block per chain -- ``loglik`` (empty: the reference
declares compute_log_likelihood but never defines it, multiview_gibbs.h:13),
``alpha_v``/``sigma_v``/``tau_v`` (list over views of float64[S]) and
``alpha_global``/``sigma_global`` (float64[S]).

The RNG is Philox4x32-10 keyed by ``seed`` instead of R's global RNG
(multiview_utils.cpp:305-306); everything runs on the GPU through
libmvc_hip.so.  Errors from the library raise ``MvcError`` (the reference
raises R conditions via Rcpp::stop, multiview_utils.cpp:141,145).
"""
import ctypes
import time
from collections.abc import Sequence

import numpy as np

from . import _lib as L


def _views_to_array(data_views):
    """List of V arrays of n (or n x D) floats -> float64 [V][n][D]."""
    if isinstance(data_views, np.ndarray):
        arr = np.asarray(data_views, dtype=np.float64)
        if arr.ndim == 2:
            arr = arr[:, :, None]
        return np.ascontiguousarray(arr)
    views = [np.asarray(v, dtype=np.float64) for v in data_views]
    if not views:
        raise ValueError("data_views must hold at least one view")
    n = views[0].shape[0]       # n is taken from view 0 (multiview_gibbs.cpp:110)
    out = []
    for v in views:
        if v.shape[0] != n:
            raise ValueError("all views must have the same number of observations")
        out.append(v.reshape(n, -1))
    D = out[0].shape[1]
    if any(v.shape[1] != D for v in out):
        raise ValueError("all views must have the same dimension")
    return np.ascontiguousarray(np.stack(out))


def _timing_flags(timing):
    """timing: False / True (every phase) / "coarse" (z-resample and whole sweeps only)."""
    if timing == "coarse":
        return L.FLAG_TIMING | L.FLAG_TIMING_COARSE
    return L.FLAG_TIMING if timing else 0


def make_config(n, V, D, M=0, burn_in=0, thin=1, seed=1999, n_chains=1, first_chain=0, device=0,
                mode="exact", table_cap=0, dish_cap=0, timing=False, quiet=True, n_devices=1, chain_stride=1):
    cfg = L.Config()
    L.lib().mvc_config_init(ctypes.byref(cfg))
    cfg.n, cfg.n_views, cfg.dim = n, V, D
    cfg.n_iter, cfg.burn_in, cfg.thin = M, burn_in, thin
    cfg.seed = seed & 0xFFFFFFFFFFFFFFFF
    cfg.n_chains, cfg.first_chain, cfg.device = n_chains, first_chain, device
    cfg.mode = {"exact": L.MODE_EXACT, "parallel": L.MODE_PARALLEL}[mode]
    cfg.table_cap, cfg.dish_cap = table_cap, dish_cap
    cfg.flags = _timing_flags(timing) | (L.FLAG_QUIET if quiet else 0)
    cfg.n_devices, cfg.chain_stride = n_devices, chain_stride
    return cfg


class _Samples(Sequence):
    """The saved samples of one chain as a read-only sequence: item s is built
    from the chain's contiguous result block when it is read (the reference's
    R list holds S small vectors per chain; materialising them eagerly for
    thousands of chains cost more than the sampling).

    table_of: `block` is the [S, n] array, item s its row s.  dish_of:
    `block` is the flat dish block, `starts` the offsets of the samples and
    `Ts` their table counts, item s the list of V rows.  Items are read-only
    views of the block; pickling (or `list(...)`) gives plain lists."""

    def __init__(self, block, starts=None, Ts=None, V=0):
        self._block = block
        self._block.flags.writeable = False
        self._starts, self._Ts, self._V = starts, Ts, V
        self._n = block.shape[0] if starts is None else len(Ts)

    def _item(self, k):
        if self._starts is None:
            return self._block[k]
        d = self._block[self._starts[k]:self._starts[k + 1]].reshape(self._V, int(self._Ts[k]))
        return [d[v] for v in range(self._V)]

    def __reduce__(self):
        return (list, (list(self),))

    def __len__(self):
        return self._n

    def __getitem__(self, s):
        if isinstance(s, slice):
            return [self._item(k) for k in range(*s.indices(self._n))]
        k = s.__index__()
        if k < 0:
            k += self._n
        if not 0 <= k < self._n:
            raise IndexError("saved sample index out of range")
        return self._item(k)

    def __repr__(self):
        return f"<{self._n} saved samples>"


def _view_ptrs(y):
    V = y.shape[0]
    arr = (ctypes.POINTER(ctypes.c_double) * V)()
    for v in range(V):
        arr[v] = y[v].ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    return arr


def run_gibbs_cpp(data_views, M, burn_in, thin, seed=1999, mode="exact", n_chains=1, device=0,
                  first_chain=0, quiet=False, n_devices=1, summary=None, timing=None):
    """Drop-in for the reference's ``run_gibbs_cpp`` (see module docstring).

    With ``n_chains > 1`` a list of per-chain result dicts is returned; the
    chains run on ``n_devices`` GPUs (chain c on device ``device + c %
    n_devices``, one host thread per device).  ``summary`` (a dict) receives
    the pooled posterior means and Gelman-Rubin R-hat of the hyperparameters
    (mvc_result_summary: keys ``mean`` and ``rhat``, float64[3V+2] in the
    order tau_v, alpha_v, sigma_v, alpha_global, sigma_global).  ``timing``
    (a dict) receives ``mvc_run_s``, the seconds of the library call alone
    (the rest is building these Python lists).
    """
    y = _views_to_array(data_views)
    V, n, D = y.shape
    cfg = make_config(n, V, D, M, burn_in, thin, seed, n_chains, first_chain, device, mode, quiet=quiet,
                      n_devices=n_devices)
    lib = L.lib()
    res = ctypes.c_void_p()
    buf = L.errbuf()
    t0 = time.perf_counter()
    L.check(lib.mvc_run(ctypes.byref(cfg), _view_ptrs(y), ctypes.byref(res), buf, len(buf)), buf)
    if timing is not None:
        timing["mvc_run_s"] = time.perf_counter() - t0
    try:
        S = lib.mvc_result_num_saved(res)
        if summary is not None:
            mean, rhat = np.empty(3 * V + 2), np.empty(3 * V + 2)
            dp = ctypes.POINTER(ctypes.c_double)
            lib.mvc_result_summary(res, mean.ctypes.data_as(dp), rhat.ctypes.data_as(dp))
            summary["mean"], summary["rhat"] = mean, rhat
        outs = []
        ip = ctypes.POINTER(ctypes.c_int32)
        for c in range(n_chains):
            # every sample of the chain in two bulk copies (mvc_result_copy_chain)
            Ts = np.zeros(S, dtype=np.int32)
            st = lib.mvc_result_copy_chain(res, c, None, Ts.ctypes.data_as(ip), None)
            if st != L.MVC_OK:
                raise L.MvcError(st, f"mvc_result_copy_chain(chain {c}) failed")
            if S > 0 and not int(Ts.sum()) > 0:
                raise L.MvcError(3, f"chain {c}: saved samples with no tables")
            tab = np.empty((S, n), dtype=np.int32)
            dsh = np.empty(max(1, V * int(Ts.sum())), dtype=np.int32)
            st = lib.mvc_result_copy_chain(res, c, tab.ctypes.data_as(ip), None, dsh.ctypes.data_as(ip))
            if st != L.MVC_OK:
                raise L.MvcError(st, f"mvc_result_copy_chain(chain {c}) failed")
            table_of = _Samples(tab)
            starts = np.concatenate(([0], np.cumsum(V * Ts.astype(np.int64))))
            dish_of = _Samples(dsh, starts, Ts, V)

            def tr(which, per_view):
                p = lib.mvc_result_trace(res, c, which)
                k = V * S if per_view else S
                a = np.ctypeslib.as_array(p, shape=(max(k, 1),))[:k].copy() if k else np.zeros(0)
                return [a[v * S:(v + 1) * S] for v in range(V)] if per_view else a

            outs.append({
                "table_of": table_of,
                "dish_of": dish_of,
                "loglik": np.zeros(0),
                "alpha_v": tr(L.TRACE_ALPHA_V, True),
                "sigma_v": tr(L.TRACE_SIGMA_V, True),
                "tau_v": tr(L.TRACE_TAU_V, True),
                "alpha_global": tr(L.TRACE_ALPHA_GLOBAL, False),
                "sigma_global": tr(L.TRACE_SIGMA_GLOBAL, False),
            })
        return outs[0] if n_chains == 1 else outs
    finally:
        lib.mvc_result_free(res)


def get_final_clusters(res):
    """Port of New_Simulation.R:135-149: per-view cluster labels of the last
    saved iteration, shape [n, V]."""
    t = res["table_of"][-1]
    dishes = res["dish_of"][-1]
    return np.stack([np.asarray(d)[t] for d in dishes], axis=1)


class Sampler:
    """Handle API: data uploaded once; sweeps run on the handle's HIP stream."""

    def __init__(self, data_views, seed=1999, mode="exact", n_chains=1, first_chain=0, device=0,
                 table_cap=0, dish_cap=0, timing=False):
        self.y = _views_to_array(data_views)
        self.V, self.n, self.D = self.y.shape
        self.n_chains = n_chains
        cfg = make_config(self.n, self.V, self.D, 0, 0, 1, seed, n_chains, first_chain, device, mode,
                          table_cap, dish_cap, timing)
        self._lib = L.lib()
        self._h = ctypes.c_void_p()
        buf = L.errbuf()
        L.check(self._lib.mvc_sampler_create(ctypes.byref(cfg), _view_ptrs(self.y), ctypes.byref(self._h), buf,
                                             len(buf)), buf)

    @classmethod
    def synthetic(cls, N, V, D, K, data_seed=1999, sd=1.3, mu_sd=3.0, seed=1999, n_chains=1, first_chain=0,
                  device=0, table_cap=0, dish_cap=0, timing=False):
        """A parallel-mode handle on synthetic data generated ON THE DEVICE
        (mvc_sampler_create_synthetic: the SURVEY §8d recipe from a Philox
        stream keyed by ``data_seed``; y never exists on the host, so N x V x D
        may exceed host memory, e.g. BASELINE configs[4] at 164 GB).  Returns
        (sampler, z) with z the generating labels (int32[N])."""
        self = cls.__new__(cls)
        self.y = None
        self.V, self.n, self.D = V, N, D
        self.n_chains = n_chains
        cfg = make_config(N, V, D, 0, 0, 1, seed, n_chains, first_chain, device, "parallel", table_cap, dish_cap,
                          timing)
        self._lib = L.lib()
        self._h = ctypes.c_void_p()
        z = np.empty(N, dtype=np.int32)
        buf = L.errbuf()
        L.check(self._lib.mvc_sampler_create_synthetic(ctypes.byref(cfg), K, ctypes.c_uint64(data_seed), sd, mu_sd,
                                                       z.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                                       ctypes.byref(self._h), buf, len(buf)), buf)
        return self, z

    def rows(self, view, idx):
        """Rows idx of view ``view`` of the handle's data (float64 [m][D]),
        read from the device (mvc_sampler_copy_rows)."""
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        out = np.empty((idx.size, self.D))
        buf = L.errbuf()
        L.check(self._lib.mvc_sampler_copy_rows(self._h, view, idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                                idx.size, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), buf,
                                                len(buf)), buf)
        return out

    def sweep(self, n_sweeps=1):
        buf = L.errbuf()
        st = self._lib.mvc_sampler_sweep(self._h, n_sweeps, buf, len(buf))
        err, self._shard_err = getattr(self, "_shard_err", None), None
        if err is not None:   # the exchange raised: the library stopped the sweep (MVC_ERR_CALLBACK)
            raise RuntimeError("shard exchange failed") from err
        L.check(st, buf)

    def synchronize(self):
        buf = L.errbuf()
        L.check(self._lib.mvc_sampler_synchronize(self._h, buf, len(buf)), buf)

    @property
    def sweeps_done(self):
        return self._lib.mvc_sampler_sweeps_done(self._h)

    def ari(self, truth, chain=0):
        """Adjusted Rand index of the chain's current table labels against
        truth[n] (mcclust::arandi, New_Simulation.R:189), on the device."""
        t = np.ascontiguousarray(truth, dtype=np.int32)
        if t.shape != (self.n,):
            raise ValueError(f"truth must have shape ({self.n},)")
        out = ctypes.c_double()
        buf = L.errbuf()
        L.check(self._lib.mvc_sampler_ari(self._h, chain, t.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                          ctypes.byref(out), buf, len(buf)), buf)
        return out.value

    def state(self, chain=0):
        """(table_of[n], dish_of[V][T], hyper dict) of one chain."""
        buf = L.errbuf()
        T = ctypes.c_int32()
        t = np.empty(self.n, dtype=np.int32)
        hy = np.empty(3 * self.V + 2)
        ip = ctypes.POINTER(ctypes.c_int32)
        dp = ctypes.POINTER(ctypes.c_double)
        L.check(self._lib.mvc_sampler_get_state(self._h, chain, t.ctypes.data_as(ip), ctypes.byref(T), None, 0,
                                                hy.ctypes.data_as(dp), buf, len(buf)), buf)
        cap = max(T.value, 1)
        d = np.empty(self.V * cap, dtype=np.int32)
        L.check(self._lib.mvc_sampler_get_state(self._h, chain, None, ctypes.byref(T), d.ctypes.data_as(ip), cap,
                                                None, buf, len(buf)), buf)
        V = self.V
        hyper = {"tau_v": hy[:V].copy(), "alpha_v": hy[V:2 * V].copy(), "sigma_v": hy[2 * V:3 * V].copy(),
                 "alpha_global": float(hy[3 * V]), "sigma_global": float(hy[3 * V + 1])}
        return t, d.reshape(V, cap)[:, :T.value].copy(), hyper

    def set_state(self, table_of, dish_of, hyper, chain=0):
        """Warm start / resume one chain (see mvc_sampler_set_state).
        table_of[n]: table positions; dish_of[V][T]: raw dish ids; hyper:
        dict as returned by state() or a flat array tau, alpha, sigma, ag, sg."""
        if isinstance(hyper, dict):
            hyper = np.concatenate([hyper["tau_v"], hyper["alpha_v"], hyper["sigma_v"],
                                    [hyper["alpha_global"], hyper["sigma_global"]]])
        t = np.ascontiguousarray(table_of, dtype=np.int32)
        d = np.ascontiguousarray(dish_of, dtype=np.int32)
        h = np.ascontiguousarray(hyper, dtype=np.float64)
        ip = ctypes.POINTER(ctypes.c_int32)
        buf = L.errbuf()
        L.check(self._lib.mvc_sampler_set_state(self._h, chain, t.ctypes.data_as(ip), d.shape[1], d.ctypes.data_as(ip),
                                                h.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), buf, len(buf)), buf)

    def dish_counts(self, chain=0):
        buf = L.errbuf()
        k = np.empty(self.V, dtype=np.int32)
        L.check(self._lib.mvc_sampler_get_dish_counts(self._h, chain, k.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                                      buf, len(buf)), buf)
        return k

    def stats(self, view, chain=0):
        """Sufficient statistics of one view: dict S1 [K][D], S2 [K], n [K]
        (live dishes in ascending raw id)."""
        buf = L.errbuf()
        K = ctypes.c_int32()
        ip = ctypes.POINTER(ctypes.c_int32)
        dp = ctypes.POINTER(ctypes.c_double)
        L.check(self._lib.mvc_sampler_get_stats(self._h, chain, view, ctypes.byref(K), None, None, None, 0, buf,
                                                len(buf)), buf)
        k = K.value
        s1 = np.empty((max(k, 1), self.D))
        s2 = np.empty(max(k, 1))
        nk = np.empty(max(k, 1), dtype=np.int32)
        L.check(self._lib.mvc_sampler_get_stats(self._h, chain, view, ctypes.byref(K), s1.ctypes.data_as(dp),
                                                s2.ctypes.data_as(dp), nk.ctypes.data_as(ip), k, buf, len(buf)), buf)
        return {"S1": s1[:k], "S2": s2[:k], "n": nk[:k]}

    def kernel_time(self, name):
        """(total_ms, launches) recorded with HIP events on the handle's stream."""
        ms = ctypes.c_double()
        cnt = ctypes.c_int64()
        st = self._lib.mvc_sampler_kernel_time(self._h, name.encode(), ctypes.byref(ms), ctypes.byref(cnt))
        if st != L.MVC_OK:
            raise L.MvcError(st, "kernel_time failed")
        return ms.value, cnt.value

    def zpath(self):
        """z-resample kernels of the last parallel sweep: bits 0-1 the lp
        producer (0 generic, 2 MFMA), bit 2 the register-resident draw kernel,
        bit 4 the all-views producer, bit 5 phase A left to the repair, bit 6
        the dish-block producer, bit 7 the row draw; -1 exact schedule / no
        sweep yet."""
        return int(self._lib.mvc_sampler_zpath(self._h))

    def phase_a(self, chain=0):
        """Phase A alone (mvc_sampler_phase_a): the next parallel sweep's
        data-parallel choices of every customer against the current state
        (table position, -1 = new table); the state is unchanged."""
        out = np.empty(self.n, dtype=np.int32)
        st = self._lib.mvc_sampler_phase_a(self._h, chain, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        if st != L.MVC_OK:
            raise L.MvcError(st, "phase_a failed")
        return out

    def repair_stats(self, chain=0):
        """Counters of the chain's last parallel sweep: dict
        moves (customers that changed table), births, rounds (in-order repair
        steps), newdish (dishes opened)."""
        out = np.zeros(4, dtype=np.int32)
        st = self._lib.mvc_sampler_repair_stats(self._h, chain, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        if st != L.MVC_OK:
            raise L.MvcError(st, "repair_stats failed")
        return dict(zip(("moves", "births", "rounds", "newdish"), (int(x) for x in out)))

    def set_shard(self, rank, world, exchange=None):
        """Within-chain N-sharding (mvc_sampler_set_shard): phase A of each
        sweep covers this rank's customers only; ``exchange`` (e.g.
        ``dist.ShardExchange``) owns the device buffer (``exchange.ptr``,
        world * shard_len int32) and its ``all_gather()`` fills every shard.
        world = 1 turns sharding off."""
        if world > 1 and exchange is None:
            raise ValueError("set_shard: world > 1 needs an exchange")
        self._shard_cb = None
        ptr = None
        if world > 1:
            def _cb(_user):
                try:
                    exchange.all_gather()
                    return 0
                except BaseException as e:   # an exception cannot cross the C frame: re-raised by sweep()
                    self._shard_err = e
                    return 1
            self._shard_cb = L.SHARD_CB(_cb)   # kept alive with the handle
            ptr = ctypes.c_void_p(exchange.ptr)
        self._shard_ex = exchange
        st = self._lib.mvc_sampler_set_shard(self._h, rank, world, ptr,
                                             ctypes.cast(self._shard_cb, ctypes.c_void_p) if self._shard_cb else None,
                                             None)
        if st != 0:
            raise L.MvcError(st, "set_shard failed")

    def set_timing(self, timing):
        """Switch HIP-event timing: False, True (every phase) or "coarse"."""
        st = self._lib.mvc_sampler_set_timing(self._h, _timing_flags(timing))
        if st != 0:
            raise RuntimeError(f"mvc_sampler_set_timing failed ({st})")

    def reset_timers(self):
        self._lib.mvc_sampler_reset_timers(self._h)

    def close(self):
        if self._h:
            self._lib.mvc_sampler_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- spec primitives on the device (parity tests) ----
def ari(a, b, device=0):
    """Adjusted Rand index of two int32 labelings (mcclust::arandi,
    the ARI of New_Simulation.R:189), computed on the device."""
    a = np.ascontiguousarray(a, dtype=np.int32)
    b = np.ascontiguousarray(b, dtype=np.int32)
    if a.shape != b.shape or a.ndim != 1:
        raise ValueError("a and b must be 1-D arrays of the same length")
    out = ctypes.c_double()
    buf = L.errbuf()
    ip = ctypes.POINTER(ctypes.c_int32)
    L.check(L.lib().mvc_ari(device, a.ctypes.data_as(ip), b.ctypes.data_as(ip), a.size, ctypes.byref(out), buf,
                            len(buf)), buf)
    return out.value


def device_math(op, x, device=0):
    ops = {"exp": 0, "log": 1, "lgamma": 2, "qnorm": 3, "sqrt": 4, "exp_sk": 5, "log_nb": 6, "exp_le0": 7, "lgamma_nb": 8}
    x = np.ascontiguousarray(x, dtype=np.float64)
    o = np.empty_like(x)
    buf = L.errbuf()
    dp = ctypes.POINTER(ctypes.c_double)
    L.check(L.lib().mvc_device_math(device, ops[op], x.ctypes.data_as(dp), o.ctypes.data_as(dp), x.size, buf,
                                    len(buf)), buf)
    return o


def device_seq_uniforms(seed, chain, start, n, device=0):
    o = np.empty(n)
    buf = L.errbuf()
    L.check(L.lib().mvc_device_seq_uniforms(device, seed, chain, start,
                                            o.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), n, buf, len(buf)), buf)
    return o


def device_tree64(x, r, device=0):
    x = np.ascontiguousarray(x, dtype=np.float64)
    rows, n = x.shape
    r = np.ascontiguousarray(r, dtype=np.float64)
    sums = np.empty(rows)
    sel = np.empty(rows, dtype=np.int64)
    buf = L.errbuf()
    dp = ctypes.POINTER(ctypes.c_double)
    L.check(L.lib().mvc_device_tree64(device, x.ctypes.data_as(dp), rows, n, r.ctypes.data_as(dp),
                                      sums.ctypes.data_as(dp), sel.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                      buf, len(buf)), buf)
    return sums, sel


def device_gemm_check(Y, S1, device=0):
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    S1 = np.ascontiguousarray(S1, dtype=np.float64)
    n, D = Y.shape
    K = S1.shape[0]
    G = np.empty((n, K))
    buf = L.errbuf()
    dp = ctypes.POINTER(ctypes.c_double)
    L.check(L.lib().mvc_device_gemm_check(device, Y.ctypes.data_as(dp), S1.ctypes.data_as(dp), n, K, D,
                                          G.ctypes.data_as(dp), buf, len(buf)), buf)
    return G
