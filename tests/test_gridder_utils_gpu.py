"""GPU parity of the gridder-utility ABI added for the w-towers path:
sdp_gridder_grid_correct_pswf / _w_stack (reference
sdp_gridder_grid_correct.h:31, :60), sdp_gridder_dft / _idft /
_image_to_flmn / _count_nonzero_pixels / _residual (reference
sdp_gridder_utils.h:54-265), each against the oracle's restatement
(oracle/wtower_oracle.py) of the reference CPU code.

Tolerances: the PSWF and pswf_n values of the library come from its own
eigen-solver (agreeing with specfun to ~1e-13), so corrections agree to
1e-12 relative in double and to one float rounding (2.5e-7) in single
precision; DFT sums differ by summation order / libm only (1e-12 double,
2e-6 single); table generators and residuals are exact.
"""
import numpy as np
import pytest

from oracle import wtower_oracle as wo

pytestmark = pytest.mark.gpu

GEO = dict(image_size=512, theta=0.02, w_step=900.0, shear_u=0.0,
           shear_v=0.0)


def _facet(rng, shape, dtype):
    x = rng.normal(size=shape)
    if np.issubdtype(dtype, np.complexfloating):
        x = x + 1j * rng.normal(size=shape)
    return x.astype(dtype)


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


@pytest.mark.parametrize("dtype,tol", [(np.float64, 1e-12),
                                       (np.complex128, 1e-12),
                                       (np.float32, 2.5e-7),
                                       (np.complex64, 2.5e-7)])
@pytest.mark.parametrize("on_device", [False, True])
def test_grid_correct_pswf(device, dtype, tol, on_device):
    import torch
    import ska_sdp_func.grid_data as g

    rng = np.random.default_rng(1)
    f = _facet(rng, (200, 160), dtype)
    ref = wo.grid_correct_pswf(GEO["image_size"], GEO["theta"],
                               GEO["w_step"], 0.0, 0.0, 8, 8, f, 30, -20)
    x = torch.from_numpy(f.copy()).to(device) if on_device else f.copy()
    g.grid_correct_pswf(GEO["image_size"], GEO["theta"], GEO["w_step"], 0.0,
                        0.0, 8, 8, x, 30, -20)
    out = x.cpu().numpy() if on_device else x
    assert _rel(out, ref) <= tol


def test_grid_correct_pswf_sheared_no_wsupport(device):
    import ska_sdp_func.grid_data as g

    rng = np.random.default_rng(2)
    f = _facet(rng, (128, 128), np.complex128)
    ref = wo.grid_correct_pswf(256, 0.01, 500.0, 0.2, 0.1, 10, 0, f, 0, 0)
    x = f.copy()
    g.grid_correct_pswf(256, 0.01, 500.0, 0.2, 0.1, 10, 0, x, 0, 0)
    assert _rel(x, ref) <= 1e-12


@pytest.mark.parametrize("dtype,tol", [(np.complex128, 1e-12),
                                       (np.complex64, 5e-7)])
@pytest.mark.parametrize("inverse", [False, True])
def test_grid_correct_w_stack(device, dtype, tol, inverse):
    import ska_sdp_func.grid_data as g
    from ska_sdp_func.utility import CError

    rng = np.random.default_rng(3)
    f = _facet(rng, (96, 128), dtype)
    ref = wo.grid_correct_w_stack(GEO["image_size"], GEO["theta"],
                                  GEO["w_step"], 0.1, 0.0, f, -40, 12, 7,
                                  inverse)
    x = f.copy()
    g.grid_correct_w_stack(GEO["image_size"], GEO["theta"], GEO["w_step"],
                           0.1, 0.0, x, -40, 12, 7, inverse)
    assert _rel(x, ref) <= tol
    y = f.copy()
    g.grid_correct_w_stack(512, 0.02, 900.0, 0.0, 0.0, y, 0, 0, 0, inverse)
    assert np.array_equal(y, f)          # w_offset 0: untouched
    with pytest.raises(CError, match="Error 3"):
        g.grid_correct_w_stack(512, 0.02, 900.0, 0.0, 0.0,
                               np.zeros((4, 4)), 0, 0, 1, inverse)


def _uvw(rng, rows, scale=3000.0):
    return rng.uniform(-scale, scale, (rows, 3))


@pytest.mark.parametrize("dbl", [True, False])
@pytest.mark.parametrize("use_chs", [False, True])
def test_dft(device, dbl, use_chs):
    import ska_sdp_func.grid_data as g

    rng = np.random.default_rng(4)
    rows, nchan, nsrc = 3000, 3, 37
    uvw = _uvw(rng, rows)
    flux = rng.uniform(0.1, 2.0, nsrc)
    lmn = np.stack([rng.uniform(-0.01, 0.01, nsrc),
                    rng.uniform(-0.01, 0.01, nsrc)], 1)
    lmn = np.concatenate([lmn, (np.sqrt(1 - (lmn ** 2).sum(1)) - 1)[:, None]],
                         1)
    s = e = None
    if use_chs:
        s = rng.integers(0, 3, rows).astype(np.int32)
        e = rng.integers(0, 4, rows).astype(np.int32)
    vis0 = (rng.normal(size=(rows, nchan))
            + 1j * rng.normal(size=(rows, nchan)))
    ut, vt, dt = ((np.float64, np.complex128, np.float64) if dbl else
                  (np.float32, np.complex64, np.float32))
    uvw_t, lmn_t = uvw.astype(ut), lmn.astype(dt)
    vis = vis0.astype(vt)
    ref = wo.dft_vis(uvw_t, s, e, flux, lmn_t.astype(np.float64), 3, -2, 1,
                     0.05, 400.0, 1.2e9, 3e6, vis)
    g.dft(uvw_t, s, e, flux, lmn_t, 3, -2, 1, 0.05, 400.0, 1.2e9, 3e6, vis)
    assert _rel(vis, ref) <= (1e-12 if dbl else 2e-6)
    if use_chs:
        skip = s >= e
        assert np.array_equal(vis[skip], vis0.astype(vt)[skip])


@pytest.mark.parametrize("dbl", [True, False])
@pytest.mark.parametrize("taper", [False, True])
def test_idft(device, dbl, taper):
    import ska_sdp_func.grid_data as g

    rng = np.random.default_rng(5)
    rows, nchan, size, theta = 400, 2, 48, 0.01
    uvw = _uvw(rng, rows)
    vt, ut = (np.complex128, np.float64) if dbl else (np.complex64,
                                                       np.float32)
    vis = (rng.normal(size=(rows, nchan))
           + 1j * rng.normal(size=(rows, nchan))).astype(vt)
    uvw_t = uvw.astype(ut)
    _, lmn = wo.image_to_flmn(np.zeros((size, size)), theta, 0.0, 0.0,
                              with_flux=False)
    lmn_t = lmn.astype(ut)
    tp = rng.uniform(0.5, 1.0, size) if taper else None
    s = rng.integers(0, 2, rows).astype(np.int32)
    e = np.full(rows, 2, np.int32)
    img0 = (rng.normal(size=(size, size)) * (1 + 1j)).astype(vt)
    ref = wo.idft_image(uvw_t, vis, s, e, lmn_t.astype(np.float64), tp, 1,
                        2, -1, theta, 300.0, 1e9, 1e7, img0)
    img = img0.copy()
    g.idft(uvw_t, vis, s, e, lmn_t, tp, 1, 2, -1, theta, 300.0, 1e9, 1e7,
           img)
    assert _rel(img, ref) <= (1e-12 if dbl else 2e-6)


@pytest.mark.parametrize("dtype,dir_t", [(np.float64, np.float64),
                                         (np.float32, np.float32),
                                         (np.complex128, np.float64),
                                         (np.complex64, np.float32),
                                         (np.complex64, np.float64)])
def test_image_to_flmn_and_count(device, dtype, dir_t):
    import torch
    import ska_sdp_func.grid_data as g

    rng = np.random.default_rng(6)
    img = np.zeros((64, 64), dtype)
    idx = rng.choice(64 * 64, 25, replace=False)
    img.ravel()[idx] = rng.uniform(0.5, 2.0, 25).astype(img.real.dtype)
    if np.issubdtype(dtype, np.complexfloating):
        img.ravel()[idx[:5]] = 1j * 0.5            # imaginary-only pixels
    n = g.count_nonzero_pixels(img)
    assert n == 25
    assert g.count_nonzero_pixels(torch.from_numpy(img).to(device)) == 25
    taper = rng.uniform(0.5, 1.0, 64)
    flux = np.zeros(n)
    lmn = np.zeros((n, 3), dir_t)
    g.image_to_flmn(img, 0.02, 0.1, -0.05, taper, flux, lmn)
    rf, rl = wo.image_to_flmn(img, 0.02, 0.1, -0.05, taper)
    np.testing.assert_array_equal(flux, rf)
    np.testing.assert_array_equal(lmn, rl.astype(dir_t))
    lmn_all = np.zeros((64 * 64, 3), dir_t)
    g.image_to_flmn(img, 0.02, 0.0, 0.0, None, None, lmn_all)
    _, ra = wo.image_to_flmn(img, 0.02, 0.0, 0.0, with_flux=False)
    np.testing.assert_array_equal(lmn_all, ra.astype(dir_t))


def test_image_to_flmn_wide_image(device):
    """A non-square image whose last columns (>= shape[0]) hold non-zero
    pixels: outputs are sized by the pixels the fill visits, an undersized
    flux array or a short taper is an argument error, not an overflow."""
    import ska_sdp_func.grid_data as g
    from ska_sdp_func.utility import CError

    img = np.zeros((16, 40))
    img[3, 5] = 1.0
    img[7, 20] = 2.0
    img[15, 39] = 3.0
    img[0, 16] = 0.5
    taper = np.linspace(0.5, 1.0, 40)
    flux = np.zeros(4)
    lmn = np.zeros((4, 3))
    g.image_to_flmn(img, 0.02, 0.0, 0.0, taper, flux, lmn)
    rf, rl = wo.image_to_flmn(img, 0.02, 0.0, 0.0, taper)
    np.testing.assert_array_equal(flux, rf)
    np.testing.assert_array_equal(lmn, rl)
    with pytest.raises(CError, match="Error 2"):
        g.image_to_flmn(img, 0.02, 0.0, 0.0, taper, np.zeros(3),
                        np.zeros((3, 3)))
    with pytest.raises(CError, match="Error 2"):
        g.image_to_flmn(img, 0.02, 0.0, 0.0, taper[:16], flux, lmn)


@pytest.mark.parametrize("ta,tb", [(np.complex128, np.complex128),
                                   (np.complex64, np.complex64),
                                   (np.complex128, np.complex64),
                                   (np.float64, np.float64),
                                   (np.float32, np.float32),
                                   (np.float64, np.float32)])
def test_residual(device, ta, tb):
    import torch
    import ska_sdp_func.grid_data as g
    from ska_sdp_func.utility import CError

    rng = np.random.default_rng(7)
    a = _facet(rng, (33, 17), ta)
    b = _facet(rng, (33, 17), tb)
    out = np.zeros_like(a)
    g.residual(torch.from_numpy(a).to(device), b, out)
    np.testing.assert_array_equal(out, a - b.astype(ta))
    with pytest.raises(CError, match="Error 6"):
        g.residual(a, b, torch.zeros((33, 17), device=device,
                                     dtype=torch.from_numpy(a).dtype))
