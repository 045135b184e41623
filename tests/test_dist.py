"""Multi-chain path on CPU: world_size 2 over gloo (the GPU run uses the same
code over RCCL).  Each rank owns one chain (dist.chain_range); the chain is
computed here by the CPU oracle (no GPU in this container); the cross-chain
hyperparameter reduce must equal the pooled statistics of both chains."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _chain(chain):
    from mvc_amd import data, dist
    from oracle import oracle as O
    y, _ = data.new_simulation(3)
    r = O.run(y, 12, 2, 1, 77, chain=chain, mode=O.PARALLEL)
    return dist.hyper_matrix(r)


def _rhat(chains):
    """Gelman-Rubin R-hat of equal-length chains (textbook formula)."""
    X = np.stack(chains)                  # [m][n][w]
    m, n = X.shape[0], X.shape[1]
    means = X.mean(axis=1)
    B = n * means.var(axis=0, ddof=1)
    W = X.var(axis=1, ddof=1).mean(axis=0)
    vplus = (n - 1) / n * W + B / n
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.where(W > 0, np.sqrt(vplus / W), np.nan)


def _worker(rank, world, port, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "multiview-clustering_amd")]
    import torch.distributed as tdist
    from mvc_amd import dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    first, nch = dist.chain_range(rank)
    H = _chain(first)
    acc = dist.HyperAccumulator(H.shape[1])
    acc.add(H)
    mean, var, cnt = acc.reduce()
    cs = dist.ChainStats(H.shape[1])
    for row in H:                 # running sums, one saved sweep at a time
        cs.add(0, row)
    r = cs.reduce()
    out[rank] = (mean, var, cnt, r["mean"], r["rhat"], r["chains"])
    tdist.barrier()
    tdist.destroy_process_group()


def test_two_rank_hyper_reduce_over_gloo():
    import torch.multiprocessing as mp
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    H = np.concatenate([_chain(0), _chain(1)])
    H0, H1 = _chain(0), _chain(1)
    rhat_ref = _rhat([H0, H1])
    for rank in range(world):
        mean, var, cnt, pmean, rhat, chains = out[rank]
        assert cnt == H.shape[0]
        assert np.allclose(mean, H.mean(axis=0), rtol=1e-12, atol=0)
        assert np.allclose(var, H.var(axis=0), rtol=1e-9, atol=1e-15)
        assert chains == 2
        assert np.allclose(pmean, H.mean(axis=0), rtol=1e-12, atol=0)
        ok = np.isfinite(rhat_ref)
        assert np.array_equal(ok, np.isfinite(rhat))
        assert np.allclose(rhat[ok], rhat_ref[ok], rtol=1e-9)
    # the two chains are genuinely different streams
    assert not np.array_equal(_chain(0), _chain(1))
