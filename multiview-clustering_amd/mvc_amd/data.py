"""Synthetic multiview data of the shapes named in BASELINE.json / SURVEY.md §8d.

All generators use numpy's PCG64 with an explicit seed (R's RNG and the
reference's own draws are not reproducible here).
Returned arrays are float64 [V][n] (D == 1) or [V][n][D].
"""
import numpy as np


def new_simulation(seed=1999, sd=1.3):
    """The data frame that New_Simulation.R:47-60 actually runs: n = 200,
    V = 5; views 1,3,4: 100 x N(3, sd) then 100 x N(-3, sd); view 2:
    50 x N(0) + 100 x N(-5) + 50 x N(5); view 5: 100 x N(-3) + 100 x N(3).
    Returns (y [5][200], true_labels list per view)."""
    rng = np.random.Generator(np.random.PCG64(seed))

    def blocks(spec):
        return np.concatenate([rng.normal(m, sd, size=k) for k, m in spec])

    two = [(100, 3.0), (100, -3.0)]
    y = np.stack([
        blocks(two),
        blocks([(50, 0.0), (100, -5.0), (50, 5.0)]),
        blocks(two),
        blocks(two),
        blocks([(100, -3.0), (100, 3.0)]),
    ])
    lab2 = np.repeat([0, 1], 100)
    lab3 = np.repeat([0, 1, 2], [50, 100, 50])
    return y, [lab2, lab3, lab2, lab2, lab2]


def config1(seed=1, n=500, sd=1.3):
    """BASELINE.json configs[0]: N = 500, V = 2, K = 3:
    view 0 three equal clusters at {-5, 0, 5}, view 1 two clusters at {-3, 3}."""
    rng = np.random.Generator(np.random.PCG64(seed))
    z = rng.integers(0, 3, size=n)
    v0 = np.array([-5.0, 0.0, 5.0])[z] + rng.normal(0, sd, size=n)
    v1 = np.array([-3.0, 3.0])[z % 2] + rng.normal(0, sd, size=n)
    return np.stack([v0, v1]), z


def synthetic(N, V, D, K, seed=0, sd=1.3, mu_sd=3.0):
    """z ~ U{0..K-1}; per-view cluster
    c_v(z) = z mod K_v with K_v = max(1, K // 2**v); means mu ~ N(0, mu_sd^2 I_D);
    y = mu[c_v(z)] + N(0, sd^2 I_D).  Returns (y [V][N][D] float64, z)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    z = rng.integers(0, K, size=N)
    y = np.empty((V, N, D), dtype=np.float64)
    for v in range(V):
        Kv = max(1, K // (2 ** v))
        mu = rng.normal(0.0, mu_sd, size=(Kv, D))
        c = z % Kv
        chunk = 1 << 18
        for a in range(0, N, chunk):
            b = min(N, a + chunk)
            y[v, a:b] = mu[c[a:b]] + rng.standard_normal((b - a, D)) * sd
    return y, z


def view_labels(z, V, K):
    """Per-view generating labels c_v(z) of `synthetic`."""
    return [z % max(1, K // (2 ** v)) for v in range(V)]
