"""bench.py's N > 1 path rehearsed on one GPU: two ranks (gloo process group,
both on device 0 through LOCAL_RANK=0), the default chains mode (one chain
per rank, chain id = rank, no collective in the sweep) and --shard (one
chain split over the ranks).  The driver's 8-GPU run launches the same code
with RCCL and one device per rank; the timing here is
meaningless, the checks are on the line rank 0 prints."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ranks(world, extra):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world),
               LOCAL_RANK="0", MVC_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--config", "c2", "--steps",
           "3", "--warmup", "1", "--no-extras", "--no-cpu-baseline"] + extra
    procs = [subprocess.Popen(cmd, env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for r in range(world - 1, -1, -1)]
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, e[-2000:]
        outs.append(o)
    lines = [ln for ln in outs[-1].strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, outs[-1][-2000:]
    for o in outs[:-1]:
        assert not [ln for ln in o.strip().splitlines() if ln.startswith("{")], "only rank 0 prints"
    return json.loads(lines[0])


def _two_ranks(extra):
    return _ranks(2, extra)


def test_bench_two_ranks_chains_mode():
    r = _two_ranks([])
    assert r["n_gpus"] == 2 and r["scaling"] == "weak"
    assert r["config"]["chains"] == 2 and r["config"]["parallelism"] == "chains2"
    # value = the sweeps of all ranks / the max-over-ranks time
    assert abs(r["value"] - 2 * r["steps"] / (r["ms_per_step"] * r["steps"] / 1e3)) <= 0.01 * r["value"]
    # the reported cross-chain reduce pooled both ranks' chains
    assert r["hyper_pooled"]["chains"] == 2
    assert r["roofline"]["bound"] in ("hbm", "mfma")


def test_bench_four_ranks_chains_mode():
    """Four ranks (the driver's 8-GPU launch has the same shape): one chain
    per rank, the line's value is all ranks' sweeps over the max-over-ranks
    time, and the pooled reduce holds four chains."""
    r = _ranks(4, [])
    assert r["n_gpus"] == 4 and r["scaling"] == "weak"
    assert r["config"]["chains"] == 4 and r["config"]["parallelism"] == "chains4"
    assert abs(r["value"] - 4 * r["steps"] / (r["ms_per_step"] * r["steps"] / 1e3)) <= 0.01 * r["value"]
    assert r["hyper_pooled"]["chains"] == 4


def test_bench_two_ranks_shard_mode():
    r = _two_ranks(["--shard"])
    assert r["n_gpus"] == 2 and r["scaling"] == "strong"
    assert r["config"]["chains"] == 1 and r["config"]["parallelism"] == "shard2"
    assert r["hyper_pooled"]["chains"] == 1
