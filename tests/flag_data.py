"""Synthetic visibilities with planted RFI for the flagger tests and bench
(test_flagger.py:19-29 scaled up)."""
import numpy as np


def make_flag_case(seed, T, B, C, P, dtype=np.complex64):
    """Complex Gaussian noise around 1+1j with planted narrowband RFI
    (strong single channels), broadband RFI (whole time steps of one
    baseline) and fluctuating channels (alternating magnitudes)."""
    rng = np.random.default_rng(seed)
    vis = (1.0 + 1.0j) + 0.05 * (rng.standard_normal((T, B, C, P))
                                 + 1j * rng.standard_normal((T, B, C, P)))
    n_nb = max(1, T * B * P // 20)
    t = rng.integers(0, T, n_nb)
    b = rng.integers(0, B, n_nb)
    c = rng.integers(0, C, n_nb)
    p = rng.integers(0, P, n_nb)
    vis[t, b, c, p] += rng.uniform(5, 40, n_nb) * np.exp(
        2j * np.pi * rng.uniform(0, 1, n_nb))
    for _ in range(max(1, B // 3)):
        tt, bb, pp = rng.integers(1, T), rng.integers(0, B), rng.integers(0, P)
        vis[tt, bb, :, pp] *= rng.uniform(3, 10)
    for _ in range(max(1, B // 2)):
        bb, cc, pp = rng.integers(0, B), rng.integers(0, C), rng.integers(0, P)
        vis[::2, bb, cc, pp] *= 2.5
    return np.ascontiguousarray(vis.astype(dtype))
