"""One rank of the within-chain N-sharding test (test_gpu_parity.py::
test_shard_ranks_equal_unsharded): ranks share one GPU, gloo exchange.

    python tests/shard_worker.py RANK WORLD PORT OUT.npz N V D K SWEEPS
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multiview-clustering_amd")]

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

import mvc_amd  # noqa: E402
from mvc_amd import data  # noqa: E402
from mvc_amd.dist import ShardExchange  # noqa: E402


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    N, V, D, K, sweeps = (int(x) for x in sys.argv[5:10])
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    y, _ = data.synthetic(N, V, D, K, seed=31)
    s = mvc_amd.Sampler(y, seed=5, mode="parallel")
    ex = ShardExchange(N, rank, world, device=0)
    s.set_shard(rank, world, ex)
    ts, hs = [], []
    for _ in range(sweeps):
        s.sweep(1)
        t, d, h = s.state()
        ts.append(t)
        hs.append(h["tau_v"])
    np.savez(out, t=np.stack(ts), d=d, tau=np.stack(hs), moves=s.repair_stats()["moves"], calls=ex.calls)
    s.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
