"""Independent chains across the GPUs of one node.

One process per GPU (torch.distributed.run); rank r runs chains
``[r * chains_per_rank, (r + 1) * chains_per_rank)`` — the chain id is part
of every Philox counter, so the streams never overlap and the sweep needs no
communication at all.  The only collective is the optional cross-chain
reduce of the hyperparameter posterior-mean accumulators (multiview_hyper.cpp
:233-292 is single-chain in the reference; pooling across chains is new):
one all-reduce of 2 (3V + 2) + 1 doubles, over RCCL (backend "nccl", a GPU
tensor) on MI355X or gloo on CPU.  The reduced values are reported, never fed
back into the chains (that would couple them and break the MCMC).

ChainStats keeps running sums per chain over the saved sweeps; its reduce
is one all-reduce of the pooled sums plus the per-chain means / variances
that the Gelman-Rubin potential scale reduction (R-hat) needs, so every rank
gets the pooled posterior means and R-hat over all chains of the node.
"""
import numpy as np

HYPER_BLOCKS = ("alpha_v", "sigma_v", "tau_v", "alpha_global", "sigma_global")


def chain_range(rank, chains_per_rank=1):
    """(first_chain, n_chains) owned by ``rank``."""
    if rank < 0 or chains_per_rank < 1:
        raise ValueError("rank >= 0 and chains_per_rank >= 1 required")
    return rank * chains_per_rank, chains_per_rank


def hyper_matrix(res):
    """Saved hyperparameter draws of one chain as float64 [S][3V+2]:
    alpha_v[0..V), sigma_v[0..V), tau_v[0..V), alpha_global, sigma_global
    (the key order of the run_gibbs_cpp result list)."""
    cols = []
    for key in HYPER_BLOCKS[:3]:
        tr = res[key]
        tr = list(tr) if isinstance(tr, (list, tuple)) else list(np.atleast_2d(tr))
        cols.extend(np.asarray(t, dtype=np.float64) for t in tr)
    cols.append(np.asarray(res["alpha_global"], dtype=np.float64))
    cols.append(np.asarray(res["sigma_global"], dtype=np.float64))
    return np.stack(cols, axis=1) if cols[0].size else np.zeros((0, len(cols)))


class HyperAccumulator:
    """Running sums of hyperparameter draws (sum, sum of squares, count)."""

    def __init__(self, width):
        self.width = int(width)
        self.s1 = np.zeros(self.width)
        self.s2 = np.zeros(self.width)
        self.count = 0

    def add(self, H):
        H = np.atleast_2d(np.asarray(H, dtype=np.float64))
        if H.shape[1] != self.width:
            raise ValueError(f"expected {self.width} hyperparameters per draw, got {H.shape[1]}")
        self.s1 += H.sum(axis=0)
        self.s2 += (H * H).sum(axis=0)
        self.count += H.shape[0]

    def packed(self):
        return np.concatenate([self.s1, self.s2, [float(self.count)]])

    def reduce(self, device=None):
        """All-reduce (sum) over the default process group; returns
        (mean, var, total_count) pooled over every rank's chains.  Without
        an initialised process group the local values are returned."""
        buf = self.packed()
        try:
            import torch
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                t = torch.from_numpy(buf.copy())
                if device is not None:
                    t = t.to(device)
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
                buf = t.cpu().numpy()
        except ImportError:
            pass
        w = self.width
        cnt = buf[-1]
        if cnt <= 0:
            return np.full(w, np.nan), np.full(w, np.nan), 0
        mean = buf[:w] / cnt
        var = np.maximum(buf[w:2 * w] / cnt - mean * mean, 0.0)
        return mean, var, int(round(cnt))


class ChainStats:
    """Running sums of each local chain's saved hyperparameter draws
    (rows of hyper_matrix: alpha_v, sigma_v, tau_v, alpha_global,
    sigma_global) for pooled posterior means and R-hat across ranks."""

    def __init__(self, width, n_chains=1):
        self.width = int(width)
        self.s1 = np.zeros((n_chains, self.width))
        self.s2 = np.zeros((n_chains, self.width))
        self.n = np.zeros(n_chains, dtype=np.int64)

    def add(self, chain, H):
        H = np.atleast_2d(np.asarray(H, dtype=np.float64))
        if H.shape[1] != self.width:
            raise ValueError(f"expected {self.width} hyperparameters per draw, got {H.shape[1]}")
        self.s1[chain] += H.sum(axis=0)
        self.s2[chain] += (H * H).sum(axis=0)
        self.n[chain] += H.shape[0]

    def packed(self):
        """[pooled s1 | pooled s2 | pooled count | sum_j mean_j | sum_j mean_j^2 |
        sum_j var_j (ddof 1) | chains | sum_j n_j]; chains with < 2 draws are
        left out of the R-hat terms."""
        w = self.width
        ok = self.n >= 2
        n = self.n[ok].astype(np.float64)[:, None]
        mean = self.s1[ok] / n if ok.any() else np.zeros((0, w))
        var = (self.s2[ok] - n * mean * mean) / (n - 1) if ok.any() else np.zeros((0, w))
        return np.concatenate([self.s1.sum(0), self.s2.sum(0), [float(self.n.sum())],
                               mean.sum(0), (mean * mean).sum(0), np.maximum(var, 0.0).sum(0),
                               [float(ok.sum()), float(self.n[ok].sum())]])

    def reduce(self, device=None):
        """All-reduce (sum) over the default process group (local values
        without one).  Returns dict(mean, var, count, chains, rhat): pooled
        mean / variance over every draw of every chain, and the Gelman-Rubin
        R-hat per hyperparameter (chains of equal length assumed; None with
        fewer than 2 chains)."""
        buf = self.packed()
        try:
            import torch
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                t = torch.from_numpy(buf.copy())
                if device is not None:
                    t = t.to(device)
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
                buf = t.cpu().numpy()
        except ImportError:
            pass
        w = self.width
        s1, s2, cnt = buf[:w], buf[w:2 * w], buf[2 * w]
        sm, smm, sv = buf[2 * w + 1:3 * w + 1], buf[3 * w + 1:4 * w + 1], buf[4 * w + 1:5 * w + 1]
        m, ntot = buf[5 * w + 1], buf[5 * w + 2]
        out = {"count": int(round(cnt)), "chains": int(round(m))}
        if cnt <= 0:
            out.update(mean=np.full(w, np.nan), var=np.full(w, np.nan), rhat=None)
            return out
        mean = s1 / cnt
        out["mean"] = mean
        out["var"] = np.maximum(s2 / cnt - mean * mean, 0.0)
        if m < 2:
            out["rhat"] = None
            return out
        n = ntot / m                                   # draws per chain
        grand = sm / m
        B = n / (m - 1) * np.maximum(smm - m * grand * grand, 0.0)   # between-chain variance
        W = sv / m                                     # mean within-chain variance
        vplus = (n - 1) / n * W + B / n
        with np.errstate(divide="ignore", invalid="ignore"):
            out["rhat"] = np.where(W > 0, np.sqrt(vplus / W), np.nan)
        return out


def shard_len(n, world):
    """Customers per shard (mvc_shard_len): ceil(n / world) rounded up to 64."""
    w = max(1, int(world))
    return ((n + w - 1) // w + 63) // 64 * 64


class ShardExchange:
    """The phase-A choice exchange of within-chain N-sharding
    (Sampler.set_shard, include/mvc.h mvc_sampler_set_shard).

    Owns a device buffer of world * shard_len(n) int32 (a torch tensor on
    this rank's GPU).  The handle copies its shard into it and calls
    all_gather() from its sweep; with backend "nccl" (RCCL over xGMI) that is
    one in-place all-gather of 4 n bytes, with "gloo" the shards go through
    host memory (tests: several ranks sharing one GPU).  Returns after the
    exchange has completed on the device."""

    def __init__(self, n, rank, world, device=0, group=None):
        import torch
        import torch.distributed as dist
        self.n, self.rank, self.world = n, rank, world
        self.S = shard_len(n, world)
        self.group = group
        self.dev = torch.device("cuda", device)
        self.buf = torch.zeros(world * self.S, dtype=torch.int32, device=self.dev)
        self.ptr = self.buf.data_ptr()
        self._dist = dist
        self._torch = torch
        self._nccl = dist.get_backend(group) == "nccl"
        self.calls = 0

    def all_gather(self):
        dist, torch = self._dist, self._torch
        self.calls += 1
        mine = self.buf[self.rank * self.S:(self.rank + 1) * self.S]
        if self._nccl:
            dist.all_gather_into_tensor(self.buf, mine, group=self.group)
            torch.cuda.synchronize(self.dev)
        else:
            host = [torch.empty(self.S, dtype=torch.int32) for _ in range(self.world)]
            dist.all_gather(host, mine.cpu(), group=self.group)
            self.buf.copy_(torch.cat(host).to(self.dev))
            torch.cuda.synchronize(self.dev)
