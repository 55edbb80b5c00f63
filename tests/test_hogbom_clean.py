"""sdp_hogbom_clean (csrc/clean/sdp_hogbom_clean.hip) against the CPU
oracle (oracle/clean_oracle.py, a restatement of sdp_hogbom_clean.cpp).

Component maps and residuals are compared bit for bit (the HIP path keeps
the reference CPU path's arithmetic: first maximum in flat order, double
products, one rounding per update); the skymodel to 1e-12 (double) /
2e-6 (float) of its peak, since the beam's exp and the convolution sum
order differ from the reference's FFT convolution by rounding. The oracle
is pinned by a delta-PSF known answer and by scipy's "same" convolution
alignment (the alignment the reference test's Python CLEAN uses).
The integration case mirrors the reference test (tests/clean/
test_hogbom_clean.py): point sources predicted with dft_point_v01 over a
random filled uv disc, dirty image and PSF made with GridderUvwEsFft,
256^2 image, 512^2 PSF, beam [2, 2, 1, 128], gain 0.1, threshold 0.001.
"""
import numpy as np
import pytest

from oracle import clean_oracle as co

BEAM = np.array([2.0, 2.0, 1.0, 128.0])


def uv_psf(n, nbl=300, seed=3):
    """[2n, 2n] PSF of a random uv disc, peak 1 at (n, n)."""
    rng = np.random.default_rng(seed)
    r = 0.4 * np.sqrt(rng.random(nbl))
    phi = 2 * np.pi * rng.random(nbl)
    u, v = r * np.cos(phi), r * np.sin(phi)
    pix = np.arange(2 * n) - n
    eu = np.exp(2j * np.pi * u[:, None] * pix[None, :])
    ev = np.exp(2j * np.pi * v[:, None] * pix[None, :])
    return (eu.T @ ev).real / nbl


def point_dirty(psf, n, nsrc=8, seed=5):
    rng = np.random.default_rng(seed)
    dirty = np.zeros((n, n))
    for _ in range(nsrc):
        x, y = rng.integers(n // 4, 3 * n // 4, 2)
        dirty += rng.uniform(1, 10) * psf[n - x:2 * n - x, n - y:2 * n - y]
    return dirty


def test_oracle_delta_psf_known_answer():
    n, g, f = 32, 0.1, 5.0
    psf = np.zeros((2 * n, 2 * n))
    psf[n, n] = 1.0
    dirty = np.zeros((n, n))
    dirty[9, 20] = f
    model, res, sky, cycles = co.hogbom_clean(dirty, psf, [1, 1, 0, 9], g,
                                              f / 2, 100)
    assert cycles == 7                       # 0.9^7 = 0.478 < 1/2 <= 0.9^6
    np.testing.assert_allclose(res[9, 20], f * 0.9 ** 7, rtol=1e-14)
    np.testing.assert_allclose(model[9, 20], f * (1 - 0.9 ** 7), rtol=1e-14)
    assert np.count_nonzero(res) == 1 and np.count_nonzero(model) == 1
    # Skymodel = component * beam centred one pixel on ((SIZE-1)//2 = 4 vs
    # centre SIZE//2 = 4 for odd SIZE: no shift) + residual.
    assert sky[9, 20] == pytest.approx(model[9, 20] + res[9, 20])
    assert sky[10, 20] == pytest.approx(model[9, 20] * np.exp(-0.5))


@pytest.mark.parametrize("nb", [8, 9, 128])
def test_oracle_restore_matches_scipy_same(nb):
    import scipy.signal as sig
    rng = np.random.default_rng(nb)
    n = 40
    model = np.zeros((n, n))
    idx = rng.integers(0, n, (12, 2))
    model[idx[:, 0], idx[:, 1]] = rng.uniform(1, 2, 12)
    beam = co.cbeam([2.5, 1.5, 30.0, nb], np.float64)
    ref = sig.convolve(model, beam, mode="same", method="direct")
    np.testing.assert_allclose(co.restore(model, beam, np.zeros((n, n))),
                               ref, atol=1e-13)


def test_library_exports_hogbom():
    from ska_sdp_func.utility import Lib
    assert hasattr(Lib.handle(), "sdp_hogbom_clean")


def _run_gpu(dirty, psf, beam, gain, thresh, cycles, device, on_device):
    from ska_sdp_func.clean import hogbom_clean
    n = dirty.shape[0]
    outs = [np.full((n, n), 9, dirty.dtype) for _ in range(3)]
    if on_device:
        import torch
        d, p = (torch.from_numpy(a).to(device) for a in (dirty, psf))
        o = [torch.from_numpy(a).to(device) for a in outs]
        hogbom_clean(d, p, beam, gain, thresh, cycles, *o)
        return [t.cpu().numpy() for t in o]
    hogbom_clean(dirty, psf, beam, gain, thresh, cycles, *outs)
    return outs


def _check(got, want, dtype):
    model, res, sky = got
    m_ref, r_ref, s_ref, _ = want
    np.testing.assert_array_equal(model, m_ref)
    np.testing.assert_array_equal(res, r_ref)
    tol = 1e-12 if dtype == np.float64 else 2e-6
    err = np.abs(sky - s_ref).max() / np.abs(s_ref).max()
    assert err < tol, err


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("on_device", [False, True])
def test_gpu_matches_oracle(device, dtype, on_device):
    # n = 200: the image is not a multiple of the workgroup span; odd beam.
    for n, beam, thresh, cycles in ((128, BEAM, 0.05, 3000),
                                    (200, [3.0, 1.5, 25.0, 33], 0.5, 500)):
        psf = uv_psf(n).astype(dtype)
        dirty = point_dirty(psf.astype(np.float64), n).astype(dtype)
        want = co.hogbom_clean(dirty, psf, beam, 0.1, thresh, cycles)
        assert 0 < want[3] <= cycles
        got = _run_gpu(dirty, psf, np.asarray(beam, dtype), 0.1, thresh,
                       cycles, device, on_device)
        _check(got, want, dtype)


@pytest.mark.gpu
def test_gpu_cycle_limit_and_threshold(device):
    n = 64
    psf = uv_psf(n)
    dirty = point_dirty(psf, n, nsrc=3)
    for thresh, cycles in ((-1.0, 37), (1e9, 10), (0.2, 64), (0.2, 65)):
        want = co.hogbom_clean(dirty, psf, BEAM, 0.2, thresh, cycles)
        got = _run_gpu(dirty, psf, BEAM, 0.2, thresh, cycles, device, True)
        _check(got, want, np.float64)


def _reference_style_data(device, n=256, nbl=2000, nsrc=10, seed=12):
    """Dirty image and PSF as the reference test builds them, on the GPU."""
    import torch
    from ska_sdp_func.grid_data import GridderUvwEsFft
    from ska_sdp_func.visibility import dft_point_v01
    rng = np.random.default_rng(seed)
    f0, df = 100e6, 100e3
    theta = 2 * np.pi * rng.random(nbl)
    radius = 3000 * rng.random(nbl)
    uvw = np.zeros((1, nbl, 3))
    uvw[0, :, 0], uvw[0, :, 1] = radius * np.cos(theta), radius * np.sin(theta)
    fluxes = np.zeros((nsrc, 1, 1), complex)
    fluxes[:, 0, 0] = rng.uniform(1, 10, nsrc)
    dirs = np.zeros((nsrc, 3))
    dirs[:, :2] = rng.uniform(-0.015, 0.015, (nsrc, 2))
    dirs[:, 2] = np.sqrt(1 - dirs[:, 0] ** 2 - dirs[:, 1] ** 2)
    images = []
    for d, f, size in ((dirs, fluxes, n),
                       (np.zeros((1, 3)), np.ones((1, 1, 1), complex), 2 * n)):
        vis = np.zeros((1, nbl, 1, 1), complex)
        dft_point_v01(d, f, uvw, f0, df, vis)
        t = [torch.from_numpy(a).to(device) for a in
             (uvw[0].copy(), np.array([f0]), vis[0].copy(),
              np.ones((nbl, 1)))]
        img = torch.zeros((size, size), dtype=torch.float64, device=device)
        px = 2 * np.pi / 180 / size
        g = GridderUvwEsFft(*t, img, px, px, 1e-5, False)
        g.grid_uvw_es_fft(*t, img)
        images.append(img.cpu().numpy() / nbl)
    return images


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_gpu_reference_style_integration(device, dtype):
    dirty, psf = (a.astype(dtype) for a in _reference_style_data(device))
    want = co.hogbom_clean(dirty, psf, BEAM, 0.1, 0.001, 10000)
    got = _run_gpu(dirty, psf, BEAM.astype(dtype), 0.1, 0.001, 10000,
                   device, True)
    _check(got, want, dtype)


@pytest.mark.gpu
def test_gpu_argument_errors(device):
    from ska_sdp_func.clean import hogbom_clean
    from ska_sdp_func.utility import CError
    n = 16
    d = np.zeros((n, n))
    outs = [np.zeros((n, n)) for _ in range(3)]
    with pytest.raises(CError, match="Generic runtime error"):
        hogbom_clean(d, np.zeros((n, n)), BEAM, 0.1, 0, 5, *outs)
    with pytest.raises(CError, match="Generic runtime error"):
        hogbom_clean(d, np.zeros((2 * n, 2 * n)), BEAM[:3], 0.1, 0, 5, *outs)
    with pytest.raises(CError, match="Generic runtime error"):
        hogbom_clean(d, np.zeros((2 * n, 2 * n)), BEAM, 0.1, 0, 0, *outs)
    with pytest.raises(CError, match="Generic runtime error"):
        hogbom_clean(d, np.zeros((2 * n, 2 * n)), BEAM, 0.0, 0, 5, *outs)
    with pytest.raises(CError, match="Unsupported data type"):
        hogbom_clean(d, np.zeros((2 * n, 2 * n), np.float32), BEAM, 0.1, 0,
                     5, *outs)
