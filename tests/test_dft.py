"""sdp_dft_point_v00 / v01 (csrc/visibility/sdp_dft.hip) against the CPU
oracle (oracle/dft_oracle.py, a restatement of sdp_dft.cpp).

The oracle is pinned by its loop form (the reference loop nest written
out scalar by scalar) and by known answers; the reference's own test
(tests/visibility/test_dft.py) only compares its CPU and GPU paths with
each other at 7 decimals and holds no golden vectors. The case shape is
the reference test's: 20 components, 4 polarisations, 10 channels,
351 baselines (27 stations), 10 times. Tolerances: complex128 1e-12
relative to the largest visibility (GPU double sincos within an ulp of
glibc's), complex64 2e-6 (same float accumulation order; the phasor
rounding can differ by one float ulp where the double sincos differ).
"""
import numpy as np
import pytest

from oracle import dft_oracle as do

F0, DF = 100e6, 10e6


def make_case(S=20, P=4, C=10, B=351, T=10, seed=4, v01=True):
    rng = np.random.default_rng(seed)
    dirs = rng.uniform(-0.1, 0.1, (S, 3))
    dirs[:, 2] = np.sqrt(1.0 - dirs[:, 0] ** 2 - dirs[:, 1] ** 2) - 1.0
    fluxes = rng.standard_normal((S, C, P)) + 1j * rng.standard_normal(
        (S, C, P))
    if v01:
        uvw = rng.uniform(-5000.0, 5000.0, (T, B, 3))
    else:
        uvw = rng.uniform(-2000.0, 2000.0, (T, B, C, 3))
    return dirs, fluxes, uvw


def oracle(dirs, fluxes, uvw, v01, shape, dtype):
    if v01:
        return do.dft_point_v01(dirs, fluxes, uvw, F0, DF, shape[2], dtype)
    return do.dft_point_v00(dirs, fluxes, uvw, dtype)


@pytest.mark.parametrize("v01", [False, True])
@pytest.mark.parametrize("dtype", [np.complex128, np.complex64])
def test_oracle_vectorised_matches_loops(v01, dtype):
    dirs, fluxes, uvw = make_case(S=5, P=4, C=3, B=4, T=2, v01=v01)
    shape = (2, 4, 3, 4)
    a = oracle(dirs, fluxes, uvw, v01, shape, dtype)
    b = do.dft_loops(dirs, fluxes, uvw, F0, DF, shape, dtype, v01)
    assert a.dtype == dtype
    np.testing.assert_array_equal(a, b)


def test_oracle_known_answers():
    # A source at the phase centre (l = m = n = 0) returns its flux.
    fluxes = np.array([[[1.5 - 2j, 0.25j]]])
    uvw = np.random.default_rng(1).uniform(-1e4, 1e4, (2, 3, 3))
    vis = do.dft_point_v01(np.zeros((1, 3)), fluxes, uvw, F0, DF, 1,
                           np.complex128)
    np.testing.assert_array_equal(vis, np.broadcast_to(fluxes[0, 0],
                                                       (2, 3, 1, 2)))
    # A unit source at l = 1 gives exp(-2 pi i u) with u in wavelengths.
    u = np.array([0.0, 0.25, 0.5, 0.125]).reshape(1, 4, 1, 1)
    uvw_l = np.concatenate([u, np.zeros((1, 4, 1, 2))], axis=-1)
    vis = do.dft_point_v00(np.array([[1.0, 0, 0]]), np.ones((1, 1, 1)),
                           uvw_l, np.complex128)
    np.testing.assert_allclose(vis[0, :, 0, 0],
                               np.exp(-2j * np.pi * u.ravel()), atol=1e-15)


def test_library_exports_dft():
    from ska_sdp_func.utility import Lib
    for name in ("sdp_dft_point_v00", "sdp_dft_point_v01"):
        assert hasattr(Lib.handle(), name)


def _tol(dtype):
    return 1e-12 if dtype == np.complex128 else 2e-6


@pytest.mark.gpu
@pytest.mark.parametrize("on_device", [False, True])
@pytest.mark.parametrize("v01", [False, True])
@pytest.mark.parametrize("dtype", [np.complex128, np.complex64])
def test_gpu_matches_oracle(device, on_device, v01, dtype):
    from ska_sdp_func.visibility import dft_point_v00, dft_point_v01
    for kw in (dict(), dict(S=300, P=1, C=3, B=700, T=2, seed=9)):
        dirs, fluxes, uvw = make_case(v01=v01, **kw)
        T, B = uvw.shape[:2]
        shape = (T, B, fluxes.shape[1], fluxes.shape[2])
        ref = oracle(dirs, fluxes, uvw, v01, shape, dtype)
        out = np.full(shape, 7 + 7j, dtype)
        arrays = [dirs, fluxes, uvw]
        if on_device:
            import torch
            arrays = [torch.from_numpy(a).to(device) for a in arrays]
            o = torch.from_numpy(out).to(device)
        else:
            o = out
        if v01:
            dft_point_v01(*arrays, F0, DF, o)
        else:
            dft_point_v00(*arrays, o)
        if on_device:
            out = o.cpu().numpy()
        err = np.abs(out - ref).max() / np.abs(ref).max()
        assert err < _tol(dtype), err


@pytest.mark.gpu
def test_gpu_empty_and_argument_errors(device):
    from ska_sdp_func.utility import CError
    from ska_sdp_func.visibility import dft_point_v00, dft_point_v01
    dirs, fluxes, uvw = make_case(S=3, P=1, C=2, B=5, T=1)
    vis = np.zeros((1, 5, 2, 1), complex)
    # No components: visibilities are written as zero.
    vis[:] = 3
    dft_point_v01(dirs[:0], fluxes[:0], uvw, F0, DF, vis)
    assert np.all(vis == 0)
    with pytest.raises(CError, match="Unsupported data type"):
        dft_point_v01(dirs, fluxes, uvw, F0, DF, np.zeros((1, 5, 2, 1)))
    with pytest.raises(CError, match="Unsupported data type"):
        dft_point_v01(dirs, fluxes.real.copy(), uvw, F0, DF, vis)
    with pytest.raises(CError, match="Invalid function argument"):
        dft_point_v01(dirs, fluxes, uvw, F0, DF,
                      np.zeros((1, 5, 2, 2), complex))
    with pytest.raises(CError, match="Unsupported data type"):
        dft_point_v01(dirs.astype(np.float32), fluxes, uvw, F0, DF, vis)
    with pytest.raises(CError):
        dft_point_v00(dirs, fluxes, uvw, vis)          # uvw must be 4D
    import torch
    with pytest.raises(CError, match="Memory location mismatch"):
        dft_point_v01(torch.from_numpy(dirs).to(device), fluxes, uvw, F0,
                      DF, vis)
