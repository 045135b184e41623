"""BASELINE config 3 data: the Reuters-21578 views of
dataset/reuters/data pre-process.R:50-108, restated by
scripts/reuters_build.py and committed as CSR counts (R's tm is absent here:
parity with tm itself is unpinned; the corpus-level counts below are the
survey's own, counted independently).  GPU: 8 chains on one MI355X."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multiview-clustering_amd")]

from mvc_amd import reuters  # noqa: E402


def test_counts_shapes_and_corpus_facts():
    body, title, topics = reuters.counts()
    N = 21578                                       # 21,578 documents
    assert body.shape[0] == title.shape[0] == topics.shape[0] == N
    assert (body.getnnz(axis=1) > 0).sum() <= 19043  # 19,043 documents with a BODY
    assert (title.getnnz(axis=1) > 0).sum() <= 20841  # 20,841 with a TITLE
    # the DTM bounds of data pre-process.R:62,81: every term in >= 5 (body) / >= 3 (title) documents
    assert (body.getnnz(axis=0) >= 5).all() and (title.getnnz(axis=0) >= 3).all()
    assert set(np.unique(topics.data)) == {1.0}     # binary <D> view (:96-102)


def test_topic_truth_top6():
    lab, names, freq = reuters.topic_truth()
    # earn 3,987, acq 2,448, money-fx 801, crude 634, grain 628, trade 552
    assert names == ["earn", "acq", "money-fx", "crude", "grain", "trade"]
    assert freq == [3987, 2448, 801, 634, 628, 552]
    assert lab.min() == -1 and lab.max() == 5
    assert np.bincount(lab[lab >= 0])[0] <= 3987


def test_views_deterministic():
    a = reuters.views()
    b = reuters.views()
    assert a.shape == (3, 21578, 64) and a.dtype == np.float64
    assert np.array_equal(a, b)
    assert np.isfinite(a).all()


def test_standardized_views():
    z = reuters.views(standardize=True)
    assert z.shape == (3, 21578, 64) and np.isfinite(z).all()
    assert np.allclose(z.mean(axis=1), 0.0, atol=1e-12)
    assert np.allclose(z.std(axis=1), 1.0, atol=1e-12)
    raw = reuters.views()
    assert float(raw[1:].std(axis=1).max()) < 0.25   # title / <D> projections: far below the N(0, 1) prior's scale


def _oracle_chain(args):
    y, chain, sweeps = args
    from oracle import oracle as O
    r = O.run(y, sweeps, 0, 1, seed=3, chain=chain, mode=O.PARALLEL)
    return r["table_of"][-1], r["dish_of"][-1], r["trace_T"]


@pytest.mark.gpu
@pytest.mark.parametrize("standardize", [False, True], ids=["raw", "standardized"])
def test_config3_full_corpus_eight_chains_one_gpu(standardize):
    """BASELINE configs[2] at its workload: the full 21,578-document corpus,
    8 concurrent chains (ChainSet) on one MI355X, one cold sweep from the
    reference initialisation (nearly every document opens a table: the
    repair's wide evaluation over ~18k tables); chains 0 and 5 equal the
    oracle's SeqSampler chains bit for bit (computed on the host meanwhile),
    and the device ARI against the top-6 TOPICS (mcclust::arandi) equals the
    oracle's for every chain."""
    from multiprocessing import get_context
    import mvc_amd
    from oracle import oracle as O
    y = np.ascontiguousarray(reuters.views(standardize=standardize))
    lab, _, _ = reuters.topic_truth()
    sel = lab >= 0
    sweeps = 1
    # the host oracle runs while the GPU sweeps, in fresh processes (a fork of
    # this process would inherit its initialised HIP runtime)
    pool = get_context("spawn").Pool(2)
    refs = pool.map_async(_oracle_chain, [(y, c, sweeps) for c in (0, 5)])
    s = mvc_amd.Sampler(y, seed=3, mode="parallel", n_chains=8)
    s.sweep(sweeps)
    s.synchronize()
    ref = dict(zip((0, 5), refs.get(timeout=600)))
    pool.close()
    for c in (0, 5):
        t, d, h = s.state(chain=c)
        assert d.shape[1] == ref[c][2][-1] > 1000, c      # thousands of tables after the cold sweep
        assert np.array_equal(t, ref[c][0]) and np.array_equal(d, ref[c][1]), c
    for c in range(8):
        t, _, _ = s.state(chain=c)
        a = mvc_amd.ari(t[sel], lab[sel])
        assert a == O.ari(t[sel], lab[sel])
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("standardize", [False, True], ids=["raw", "standardized"])
def test_config3_prefix_two_sweeps(standardize):
    """The first 2,000 documents, 8 chains, two cold sweeps: chains 0 and 5
    bit for bit vs the oracle's SeqSampler."""
    import mvc_amd
    from oracle import oracle as O
    n = 2000
    y = np.ascontiguousarray(reuters.views(standardize=standardize)[:, :n])
    s = mvc_amd.Sampler(y, seed=3, mode="parallel", n_chains=8)
    s.sweep(2)
    for c in (0, 5):
        ref = O.run(y, 2, 0, 1, seed=3, chain=c, mode=O.PARALLEL)
        t, d, h = s.state(chain=c)
        assert np.array_equal(t, ref["table_of"][-1]) and np.array_equal(d, ref["dish_of"][-1]), c
    s.close()
