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
    out[rank] = (mean, var, cnt)
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
    for rank in range(world):
        mean, var, cnt = out[rank]
        assert cnt == H.shape[0]
        assert np.allclose(mean, H.mean(axis=0), rtol=1e-12, atol=0)
        assert np.allclose(var, H.var(axis=0), rtol=1e-9, atol=1e-15)
    # the two chains are genuinely different streams
    assert not np.array_equal(_chain(0), _chain(1))
