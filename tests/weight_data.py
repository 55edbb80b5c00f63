"""Inputs for the weighting tests.

`prime_case` and `flat_case` carry the input arrays of the reference's own
test module (tests/visibility/test_weighting.py: prime_3x3_input,
gpu_input) as data; `random_case` is synthetic, with a share of the
visibilities off the grid (|u| or |v| beyond max_abs_uv, or negative cell
indices)."""
import numpy as np

MAX_ABS_UV_REF = 16011.076569511299   # the reference tests' control value


def prime_case():
    freqs = np.array([1e9, 1.1e9, 1.2e9])
    uvw = np.array([[[2, 3, 5], [7, 11, 13], [17, 19, 23]]], np.float64)
    w = np.array([10.0, 31.0, 21.0])
    inp = np.broadcast_to(w[None, None, :, None], (1, 3, 3, 1)).copy()
    return freqs, uvw, MAX_ABS_UV_REF, inp


def flat_case():
    freqs = 1e9 + 1e8 * np.arange(6)
    uvw = np.broadcast_to(np.array([10.0, 31.0, 21.0]), (8, 8, 3)).copy()
    w = np.array([24.0, 38.0, 47.0, 81.0, 21.0, 41.0])
    inp = np.broadcast_to(w[None, None, :, None], (8, 8, 6, 1)).copy()
    return freqs, uvw, MAX_ABS_UV_REF, inp


def random_case(T=20, B=50, C=8, P=2, seed=3, dtype=np.float64):
    rng = np.random.default_rng(seed)
    freqs = 1e9 + 2e7 * np.arange(C)
    uvw = rng.normal(0.0, 3000.0, (T, B, 3))
    inp = rng.uniform(0.5, 2.0, (T, B, C, P)).astype(dtype)
    # About 15 % of the visibilities fall off the grid (|u f / c| beyond it).
    max_abs_uv = 0.8 * float(np.max(np.abs(uvw[:, :, :2]))) * freqs[-1] \
        / 299792458.0
    return freqs, uvw, max_abs_uv, inp
