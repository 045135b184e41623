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
