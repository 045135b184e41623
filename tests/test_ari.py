"""ARI (the caller's mcclust::arandi, New_Simulation.R:5,189).

CPU: the oracle restatement pinned against scikit-learn's adjusted_rand_score
(the same Hubert-Arabie index; mcclust itself is an R package absent here) and
known answers, including arandi's NaN for a 1 x 1 table.  GPU: the device ARI (C ABI) equals the oracle bit for bit,
including on a sampler's own state."""
import numpy as np
import pytest

from oracle import oracle as O


def _cases():
    rng = np.random.default_rng(7)
    yield rng.integers(0, 5, 1000), rng.integers(0, 7, 1000)
    z = rng.integers(0, 16, 20000)
    noisy = np.where(rng.random(20000) < 0.2, rng.integers(0, 16, 20000), z)
    yield z, noisy
    yield rng.integers(-3, 3, 257), rng.integers(100, 140, 257)        # negative / offset labels
    yield np.arange(50), rng.integers(0, 2, 50)                        # all singletons vs two blocks
    yield np.zeros(10, int), rng.integers(0, 3, 10)                    # one block vs three


def test_oracle_ari_matches_sklearn():
    from sklearn.metrics import adjusted_rand_score
    for a, b in _cases():
        assert np.isclose(O.ari(a, b), adjusted_rand_score(a, b), rtol=1e-12, atol=1e-15)


def test_oracle_ari_known_answers():
    a = np.array([0, 0, 1, 1, 2, 2])
    assert O.ari(a, a) == 1.0
    assert O.ari(a, 5 - a) == 1.0                     # label permutation
    assert np.isnan(O.ari(np.zeros(7, int), np.ones(7, int)))   # arandi: 1 x 1 table is 0/0
    # two 3-cluster labelings of 6 items: a = 2, sa = 6, sb = 3, C(6,2) = 15,
    # correc = 18/15 = 1.2, (2 - 1.2) / (4.5 - 1.2) in R's fp64 order
    assert O.ari([0, 0, 0, 1, 1, 1], [0, 0, 1, 1, 2, 2]) == (2.0 - 18.0 / 15.0) / ((0.5 * 6 + 0.5 * 3) - 18.0 / 15.0)
    assert np.isclose(O.ari([0, 0, 0, 1, 1, 1], [0, 0, 1, 1, 2, 2]), 0.24242424242424243)


@pytest.mark.gpu
def test_device_ari_bitwise_vs_oracle():
    import mvc_amd
    for a, b in _cases():
        assert mvc_amd.ari(a, b) == O.ari(a, b)
    assert np.isnan(mvc_amd.ari(np.zeros(9, int), np.full(9, 4)))   # arandi: 1 x 1 table
    rng = np.random.default_rng(3)
    a = rng.integers(0, 64, 1_000_000)
    b = np.where(rng.random(a.size) < 0.1, rng.integers(0, 64, a.size), a % 16)
    assert mvc_amd.ari(a, b) == O.ari(a, b)
    a = rng.integers(0, 3000, 200_000)                  # table beyond LDS: global-atomic path
    b = rng.integers(0, 500, 200_000)
    assert mvc_amd.ari(a, b) == O.ari(a, b)
    with pytest.raises(mvc_amd.MvcError):
        mvc_amd.ari(np.array([0, 1 << 20]), np.array([0, 1 << 20]))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["parallel", "exact"])
def test_sampler_ari_vs_state(mode):
    import mvc_amd
    from mvc_amd import data
    n, D = (20000, 8) if mode == "parallel" else (600, 1)    # exact mode: the reference's scalar views
    y, z = data.synthetic(n, 2, D, 8, seed=9)
    s = mvc_amd.Sampler(y, seed=5, mode=mode)
    s.sweep(3)
    t, _, _ = s.state()
    assert s.ari(z) == O.ari(t, z)
    s.close()
