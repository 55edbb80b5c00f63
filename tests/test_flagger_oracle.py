"""CPU tests of the flagger oracle (oracle/flagger_oracle.c).

Pinned by the reference's own known-answer test
(tests/visibility/test_flagger.py:11-65 of ska-sdp-func 1.2.2): same data,
parameters and expected mask, restated here as data.
"""
import numpy as np
import pytest

from oracle import flagger_oracle as fo


def reference_fixture(dtype=np.complex128):
    """test_flagger.py:11-29: 50 x 3 x 100 x 4, planted RFI."""
    vis = np.zeros((50, 3, 100, 4), dtype=dtype)
    vis[:, :, :, :] = complex(1, 1)
    vis[10, 0, 28, :] = 20 + 4j
    vis[36, 0, 14, 0] = vis[36, 0, 14, 0] + 0.08 + 0.08j
    vis[27, 1, :, 2] = 20 + 30j
    expected = np.zeros(vis.shape, dtype=np.int32)
    expected[9, 0, 28, :] = 1
    expected[10, 0, 28, :] = 1
    expected[11, 0, 28, :] = 1
    expected[36, 0, 14, 0] = 1
    expected[27, 1, :, 2] = 1
    return vis, expected


REF_ARGS = dict(alpha=0.5, threshold_magnitudes=3.5, threshold_variations=3.5,
                threshold_broadband=3.5, sampling_step=1, window=0,
                window_median_history=20)


@pytest.mark.parametrize("dtype", [np.complex128, np.complex64])
def test_reference_known_answer(dtype):
    vis, expected = reference_fixture(dtype)
    flags = np.zeros(vis.shape, np.int32)
    fo.flagger_dynamic_threshold(vis, flags, **REF_ARGS)
    assert np.array_equal(flags, expected)


def test_flags_only_set_never_cleared():
    vis, expected = reference_fixture()
    flags = np.zeros(vis.shape, np.int32)
    flags[0, 2, 5, 1] = 1
    fo.flagger_dynamic_threshold(vis, flags, **REF_ARGS)
    want = expected.copy()
    want[0, 2, 5, 1] = 1
    assert np.array_equal(flags, want)


def test_window_never_flags_channel_zero():
    """sdp_flagger.cpp:232: neighbours need c - w - 1 > 0."""
    vis, _ = reference_fixture()
    vis[:] = 1 + 1j
    vis[20, 0, 1, 0] = 40 + 0j          # channel 1: neighbour 0 and 2
    flags = np.zeros(vis.shape, np.int32)
    args = dict(REF_ARGS, window=1)
    fo.flagger_dynamic_threshold(vis, flags, **args)
    assert flags[20, 0, 2, 0] == 1 and flags[20, 0, 1, 0] == 1
    assert flags[20, 0, 0, 0] == 0


def _hypot_glibc_kernel(x, y):
    """Vectorised restatement of the device |v| for complex128
    (csrc/visibility/sdp_flagger.hip: glibc 2.35 e_hypot.c, non-FMA
    kernel), for finite inputs in the unscaled range."""
    x, y = np.abs(x), np.abs(y)
    ax, ay = np.maximum(x, y), np.minimum(x, y)
    h = np.sqrt(ax * ax + ay * ay)
    big = h <= 2.0 * ay
    d1 = h - ay
    t1a = ax * (2.0 * d1 - ax)
    t2a = (d1 - 2.0 * (ax - ay)) * d1
    d2 = h - ax
    t1b = 2.0 * d2 * (ax - 2.0 * ay)
    t2b = (4.0 * d2 - ay) * ay + d2 * d2
    t1 = np.where(big, t1a, t1b)
    t2 = np.where(big, t2a, t2b)
    r = h - (t1 + t2) / (2.0 * h)
    return np.where(ay <= ax * 2.0 ** -54, ax + ay, r)


def test_device_magnitude_formulas_match_glibc():
    """The reference's |v| is glibc cabsf / cabs (std::abs of
    std::complex). The device reproduces them as (float)sqrt(x^2 + y^2) in
    double (cabsf) and glibc's hypot kernel (cabs); both checked here on
    10^6 values against the oracle's glibc calls."""
    rng = np.random.default_rng(0)
    n = 1_000_000
    v = (rng.standard_normal(n) * 10.0 ** rng.uniform(-6, 6, n)
         + 1j * rng.standard_normal(n) * 10.0 ** rng.uniform(-6, 6, n))
    x = v.astype(np.complex64)
    re, im = x.real.astype(np.float64), x.imag.astype(np.float64)
    f32 = np.sqrt(re * re + im * im).astype(np.float32).astype(np.float64)
    assert np.array_equal(fo.cabs(x), f32)
    x = v.astype(np.complex128)
    assert np.array_equal(fo.cabs(x), _hypot_glibc_kernel(x.real, x.imag))
