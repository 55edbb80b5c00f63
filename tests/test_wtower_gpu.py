"""GPU parity of the HIP w-towers gridder (csrc/grid_data/
sdp_gridder_wtower_uvw.hip, sdp_gridder_utils.hip, sdp_gridder_wtower_
height.hip) with the oracle (oracle/wtower_oracle.py).

The oracle restates sdp_gridder_wtower_uvw.cpp and its helpers in float64
and is pinned by the DFT and the grid/degrid adjoint identity
(tests/test_wtower_oracle.py). Tolerances: complex128 paths agree with the
oracle to 1e-10 of the largest value (FFT libraries and summation order
differ; the arithmetic is otherwise the reference's); complex64 paths to
2e-5 (single-precision stack, as the reference's c64 path).
"""
import ctypes

import numpy as np
import pytest

import wtower_data as wd
from oracle import wtower_oracle as wo

pytestmark = pytest.mark.gpu

C0 = wd.C_0
TOL = {np.complex128: 1e-10, np.complex64: 2e-5}


def _plan(cfg=None):
    from ska_sdp_func.grid_data import GridderWtowerUVW
    cfg = cfg or wd.REF_CFG
    return GridderWtowerUVW(**cfg), wo.WtowerPlan(**cfg)


def _to(x, device):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x)).to(device)


def _close(a, b, tol):
    scale = max(np.abs(b).max(), 1e-300)
    err = np.abs(a - b).max() / scale
    assert err <= tol, f"max rel err {err:.3e} > {tol:.1e}"


def _ref_inputs(num_chan=2, seed=0, uvw_dtype=np.float64):
    uvw = wd.generate_uvw().astype(uvw_dtype)
    R = uvw.shape[0]
    rng = np.random.default_rng(seed)
    sc = rng.integers(0, num_chan, R).astype(np.int32)
    sc[::5] = 0
    ec = np.full(R, num_chan, np.int32)
    ec[::7] = sc[::7]          # some empty rows
    return uvw, sc, ec


CASES = [
    # (vis dtype, uvw dtype)
    (np.complex128, np.float64),
    (np.complex64, np.float64),
    (np.complex64, np.float32),
]


@pytest.mark.parametrize("vis_t,uvw_t", CASES)
@pytest.mark.parametrize("on_device", [False, True])
def test_degrid_matches_oracle(device, vis_t, uvw_t, on_device):
    gp, op = _plan()
    uvw, sc, ec = _ref_inputs(3, uvw_dtype=uvw_t)
    R = uvw.shape[0]
    rng = np.random.default_rng(4)
    img = wd.ref_image().astype(vis_t)
    img += (0.01 * rng.normal(size=img.shape)).astype(vis_t)
    vis0 = (rng.normal(size=(R, 3)) + 1j * rng.normal(size=(R, 3))).astype(
        vis_t)
    ref = op.degrid(img.astype(np.complex128), *wd.REF_OFFSETS, C0, C0 / 100,
                    uvw, sc, ec, vis0.astype(np.complex128))
    if on_device:
        v = _to(vis0, device)
        gp.degrid(_to(img, device), *wd.REF_OFFSETS, C0, C0 / 100,
                  _to(uvw, device), _to(sc, device), _to(ec, device), v)
        out = v.cpu().numpy()
    else:
        out = vis0.copy()
        gp.degrid_subgrid(img, wd.REF_OFFSETS, 3, C0, C0 / 100, uvw, sc, ec,
                          out)
    _close(out - vis0, ref - vis0, TOL[vis_t])
    assert gp.num_w_planes(False) == op.num_w_planes[0] > 100


@pytest.mark.parametrize("vis_t,uvw_t", CASES)
@pytest.mark.parametrize("on_device", [False, True])
def test_grid_matches_oracle(device, vis_t, uvw_t, on_device):
    gp, op = _plan()
    uvw, sc, ec = _ref_inputs(3, seed=1, uvw_dtype=uvw_t)
    R = uvw.shape[0]
    rng = np.random.default_rng(5)
    vis = (rng.normal(size=(R, 3)) + 1j * rng.normal(size=(R, 3))).astype(
        vis_t)
    img0 = (rng.normal(size=(64, 64)) + 1j * rng.normal(size=(64, 64))
            ).astype(vis_t)
    ref = op.grid(vis.astype(np.complex128), uvw, sc, ec, C0, C0 / 100,
                  img0.astype(np.complex128), *wd.REF_OFFSETS)
    if on_device:
        img = _to(img0, device)
        gp.grid(_to(vis, device), _to(uvw, device), _to(sc, device),
                _to(ec, device), C0, C0 / 100, img, *wd.REF_OFFSETS)
        out = img.cpu().numpy()
    else:
        out = img0.copy()
        gp.grid_subgrid(vis, uvw, sc, ec, 3, C0, C0 / 100, out,
                        wd.REF_OFFSETS)
    _close(out - img0, ref - img0, TOL[vis_t])


def test_row_range_and_real_image(device):
    """start_row / end_row restrict the rows; a real sub-grid image takes
    the real part of the gridded result (accumulate_scaled_arrays)."""
    gp, op = _plan()
    uvw, sc, ec = _ref_inputs(2, seed=2)
    R = uvw.shape[0]
    rng = np.random.default_rng(6)
    vis = rng.normal(size=(R, 2)) + 1j * rng.normal(size=(R, 2))
    img = np.zeros((64, 64))
    gp.grid(vis, uvw, sc, ec, C0, C0 / 100, img, *wd.REF_OFFSETS, 1000, 5000)
    ref = op.grid(vis, uvw, sc, ec, C0, C0 / 100, np.zeros((64, 64)),
                  *wd.REF_OFFSETS, 1000, 5000)
    _close(img, ref, 1e-10)
    out = np.zeros((R, 2), np.complex128)
    gp.degrid(wd.ref_image(), *wd.REF_OFFSETS, C0, C0 / 100, uvw, sc, ec,
              out, 1000, 5000)
    ref = op.degrid(wd.ref_image().astype(complex), *wd.REF_OFFSETS, C0,
                    C0 / 100, uvw, sc, ec, np.zeros((R, 2), complex), 1000,
                    5000)
    _close(out, ref, 1e-10)
    assert not out[:1000].any() and not out[5000:].any()


def test_subgrid_edge_wraps_like_reference(device):
    """Visibilities within support / 2 of the sub-grid edge address the
    stack past a layer's end; the result follows the reference's flat
    indexing (oracle), and nothing outside the stack is touched."""
    cfg = dict(wd.REF_CFG, theta=0.01)
    gp, op = _plan(cfg)
    rng = np.random.default_rng(9)
    R = 400
    half = 32 / 0.01
    uvw = np.zeros((R, 3))
    uvw[:, 0] = rng.uniform(-half, half, R)
    uvw[:, 1] = rng.uniform(-half, half, R)
    uvw[:, 2] = rng.uniform(-2000, 2000, R)
    sc = np.zeros(R, np.int32)
    ec = np.ones(R, np.int32)
    img = rng.normal(size=(64, 64)) + 1j * rng.normal(size=(64, 64))
    out = np.zeros((R, 1), complex)
    gp.degrid(img, 0, 0, 0, C0, C0 / 100, uvw, sc, ec, out)
    ref = op.degrid(img, 0, 0, 0, C0, C0 / 100, uvw, sc, ec,
                    np.zeros((R, 1), complex))
    _close(out, ref, 1e-10)
    vis = rng.normal(size=(R, 1)) + 1j * rng.normal(size=(R, 1))
    sub = np.zeros((64, 64), complex)
    gp.grid(vis, uvw, sc, ec, C0, C0 / 100, sub, 0, 0, 0)
    ref = op.grid(vis, uvw, sc, ec, C0, C0 / 100, np.zeros((64, 64), complex),
                  0, 0, 0)
    _close(sub, ref, 1e-10)


def test_large_subgrid_adjoint(device):
    """Size-independent check at a cfg4-like sub-grid (S = 256): gridding is
    the adjoint of degridding on the GPU, in both precisions."""
    import torch
    from ska_sdp_func.grid_data import GridderWtowerUVW
    S, theta = 256, 0.02
    gp = GridderWtowerUVW(4096, S, theta, 500.0, 0.1, -0.05, 8, 16384, 8,
                          16384)
    rng = np.random.default_rng(11)
    R, C = 20000, 4
    lim = 0.4 * S / theta
    uvw = np.stack([rng.uniform(-lim, lim, R), rng.uniform(-lim, lim, R),
                    rng.uniform(-20000, 20000, R)], axis=1)
    sc = np.zeros(R, np.int32)
    ec = np.full(R, C, np.int32)
    for vis_t, tol in [(np.complex128, 1e-11), (np.complex64, 1e-4)]:
        x = (rng.normal(size=(S, S)) + 1j * rng.normal(size=(S, S))).astype(
            vis_t)
        y = (rng.normal(size=(R, C)) + 1j * rng.normal(size=(R, C))).astype(
            vis_t)
        ax = torch.zeros((R, C), dtype=torch.complex128 if vis_t is
                         np.complex128 else torch.complex64, device=device)
        d_uvw = _to(uvw, device)
        d_sc, d_ec = _to(sc, device), _to(ec, device)
        gp.degrid(_to(x, device), 0, 0, 0, C0, C0 / 1000, d_uvw, d_sc, d_ec,
                  ax)
        gy = torch.zeros((S, S), dtype=ax.dtype, device=device)
        gp.grid(_to(y, device), d_uvw, d_sc, d_ec, C0, C0 / 1000, gy, 0, 0, 0)
        lhs = np.vdot(y.astype(np.complex128),
                      ax.cpu().numpy().astype(np.complex128))
        rhs = np.vdot(gy.cpu().numpy().astype(np.complex128),
                      x.astype(np.complex128))
        assert abs(lhs - rhs) <= tol * abs(lhs)
    assert gp.num_w_planes(False) > 50


@pytest.mark.parametrize("dtype", [np.float64, np.complex128, np.float32,
                                   np.complex64])
@pytest.mark.parametrize("w_offset", [0, 50, -3])
def test_correct_matches_oracle(device, dtype, w_offset):
    cfg = dict(wd.REF_CFG, theta=0.1)
    gp, op = _plan(cfg)
    rng = np.random.default_rng(12)
    facet = rng.random((64, 64))
    if np.iscomplexobj(np.zeros(1, dtype)):
        facet = facet + 1j * rng.random((64, 64))
    facet = facet.astype(dtype)
    tol = 1e-12 if dtype in (np.float64, np.complex128) else 1e-6
    for inverse in (False, True):
        out = facet.copy()
        ref = facet.astype(np.complex128 if np.iscomplexobj(facet)
                           else np.float64)
        if inverse:
            gp.grid_correct(out, 5, -15, w_offset)
            op.grid_correct(ref, 5, -15, w_offset)
        else:
            gp.degrid_correct(out, 5, -15, w_offset)
            op.degrid_correct(ref, 5, -15, w_offset)
        _close(out, ref, tol)


def test_correct_on_device(device):
    cfg = dict(wd.REF_CFG, theta=0.1)
    gp, op = _plan(cfg)
    facet = np.random.default_rng(13).random((64, 64)) + 0j
    d = _to(facet, device)
    gp.degrid_correct(d, 5, -15, 50)
    _close(d.cpu().numpy(), op.degrid_correct(facet.copy(), 5, -15, 50),
           1e-12)


# -- utilities ---------------------------------------------------------------

def test_subgrid_cut_out_and_add(device):
    import ska_sdp_func.grid_data as g
    rng = np.random.default_rng(123)
    grid = rng.random((512, 512)) + 0j
    sub = np.zeros((128, 128), np.complex128)
    g.subgrid_cut_out(grid, -255, -170, sub)
    np.testing.assert_array_equal(sub, wo.subgrid_cut_out(grid, -255, -170,
                                                          128, 128))
    sub = rng.random((128, 128)) + 0j
    out = np.zeros((512, 512), np.complex128)
    g.subgrid_add(out, -255, -170, sub, 16.0)
    ref = np.zeros((512, 512), np.complex128)
    wo.subgrid_add(ref, -255, -170, sub, 16.0)
    np.testing.assert_array_equal(out, ref)
    d_out = _to(np.zeros((512, 512), np.float32), device)
    g.subgrid_add(d_out, 7, 9, _to(sub.real.astype(np.float32), device), 2.0)
    ref = np.zeros((512, 512))
    wo.subgrid_add(ref, 7, 9, sub.real.astype(np.float32).astype(np.float64),
                   2.0)
    np.testing.assert_allclose(d_out.cpu().numpy(), ref, rtol=1e-7)


@pytest.mark.parametrize("uvw_t", [np.float64, np.float32])
def test_uvw_bounds_and_clamp(device, uvw_t):
    import ska_sdp_func.grid_data as g
    uvw, sc, ec = _ref_inputs(16, seed=3, uvw_dtype=uvw_t)
    lo, hi = g.uvw_bounds_all(uvw, C0, C0 / 100, sc, ec)
    rlo, rhi = wo.uvw_bounds_all(uvw, C0, C0 / 100, sc, ec)
    np.testing.assert_allclose(list(lo), rlo, rtol=1e-15)
    np.testing.assert_allclose(list(hi), rhi, rtol=1e-15)
    so = np.zeros_like(sc)
    eo = np.zeros_like(ec)
    g.clamp_channels_single(uvw, 1, C0, C0 / 100, sc, ec, -3000.0, 5000.0,
                            so, eo)
    rs, re_ = wo.clamp_channels_rows(uvw, 1, C0, C0 / 100, sc, ec, -3000.0,
                                     5000.0)
    np.testing.assert_array_equal(so, rs)
    np.testing.assert_array_equal(eo, re_)
    so[:] = -1
    eo[:] = -1
    g.clamp_channels_uv(_to(uvw, device), C0, C0 / 100, _to(sc, device),
                        _to(ec, device), -8000.0, 2000.0, -1000.0, 9000.0,
                        d_so := _to(so, device), d_eo := _to(eo, device),
                        100, 9000)
    rs, re_ = wo.clamp_channels_uv_rows(uvw, C0, C0 / 100, sc, ec, -8000.0,
                                        2000.0, -1000.0, 9000.0, 100, 9000)
    so, eo = d_so.cpu().numpy(), d_eo.cpu().numpy()
    np.testing.assert_array_equal(so[100:9000], rs[100:9000])
    np.testing.assert_array_equal(eo[100:9000], re_[100:9000])
    assert (so[:100] == -1).all() and (eo[9000:] == -1).all()


def _c_api():
    from ska_sdp_func.utility import Lib, Mem
    M = Mem.handle_type()
    Lib.wrap_func("sdp_gridder_sum_diff", restype=None,
                  argtypes=[M, M, ctypes.POINTER(ctypes.c_int64),
                            ctypes.c_int64, ctypes.c_int64],
                  check_errcode=True)
    Lib.wrap_func("sdp_gridder_scale_inv_array", restype=None,
                  argtypes=[M, M, M, ctypes.c_int], check_errcode=True)
    Lib.wrap_func("sdp_gridder_accumulate_scaled_arrays", restype=None,
                  argtypes=[M, M, M, ctypes.c_int], check_errcode=True)
    Lib.wrap_func("sdp_gridder_shift_subgrids", restype=None,
                  argtypes=[M], check_errcode=True)
    return Lib, Mem


def test_array_utilities(device):
    Lib, Mem = _c_api()
    rng = np.random.default_rng(21)
    a = rng.integers(-1000, 1000, 5000).astype(np.int32)
    b = rng.integers(-1000, 1000, 5000).astype(np.int32)
    res = ctypes.c_int64(0)
    Lib.sdp_gridder_sum_diff(Mem(a), Mem(b), ctypes.byref(res), 10, 4000)
    assert res.value == int(a[10:4000].astype(np.int64).sum()
                            - b[10:4000].astype(np.int64).sum())
    w = wo.make_w_pattern(64, 0.0008, 0.2, 0.1, 280.0)
    x = rng.normal(size=(64, 64)) + 1j * rng.normal(size=(64, 64))
    for e in (1, 5, -7, 0):
        out = np.zeros_like(x)
        Lib.sdp_gridder_scale_inv_array(Mem(out), Mem(x), Mem(w), e)
        _close(out, x / w ** e, 1e-14)
        acc = x.copy()
        Lib.sdp_gridder_accumulate_scaled_arrays(Mem(acc), Mem(x), Mem(w), e)
        _close(acc, x + x * w ** e, 1e-14)
    real = np.zeros((64, 64))
    Lib.sdp_gridder_accumulate_scaled_arrays(Mem(real), Mem(x), Mem(w), 3)
    np.testing.assert_array_equal(real, x.real)   # real out: in2 ignored
    stack = rng.normal(size=(5, 64, 64)) + 0j
    d = _to(stack, device)
    Lib.sdp_gridder_shift_subgrids(Mem(d))
    np.testing.assert_array_equal(d.cpu().numpy()[:4], stack[1:])
    np.testing.assert_array_equal(d.cpu().numpy()[4], stack[4])
    import ska_sdp_func.grid_data as g
    y = x + 1e-3
    assert abs(g.rms_diff(x, y) - 1e-3) < 1e-15


def test_determine_max_w_tower_height(device):
    import ska_sdp_func.grid_data as g
    args = (256, 128, 0.01, wo.determine_w_step(0.01, 0.008, 0.0, 0.0), 0.0,
            0.0, 10, 16384, 10, 16384, 0.008)
    ref = wo.determine_max_w_tower_height(*args)
    got = g.determine_max_w_tower_height(
        128, 0.01, 0.008, args[3], 10, 16384, 10, 16384, image_size=256,
        subgrid_frac=0.0, num_samples=0)
    assert got == ref == 18.0


def test_argument_errors(device):
    from ska_sdp_func.utility import CError
    gp, _ = _plan()
    uvw, sc, ec = _ref_inputs(2)
    R = uvw.shape[0]
    img = np.zeros((64, 64), np.complex128)
    with pytest.raises(CError, match="Memory location"):
        gp.degrid(img, 0, 0, 0, C0, C0 / 100, _to(uvw, device), sc, ec,
                  np.zeros((R, 2), np.complex128))
    with pytest.raises(CError, match="data type"):
        gp.degrid(img, 0, 0, 0, C0, C0 / 100, uvw, sc, ec,
                  np.zeros((R, 2), np.float64))
    with pytest.raises(CError, match="data type"):
        gp.degrid(img.astype(np.complex64), 0, 0, 0, C0, C0 / 100, uvw, sc,
                  ec, np.zeros((R, 2), np.complex128))


def test_reference_python_test_tolerances_c128(device):
    """The reference Python test's own bounds for its C++-vs-NumPy check,
    applied to the HIP kernels against the oracle in complex double:
    degridded visibilities per row atol 1e-14, rtol 1e-13
    (test_gridder_wtower_uvw.py:1642-1651). For gridding the reference
    bounds max |diff| < 1e-10 (:1688) on a sub-grid that its offsets place
    beyond every baseline, so its images are zero (wtower_data.REF_OFFSETS);
    on these offsets the image peak is ~360 and the bound is applied
    relative to it, at 2e-12 (measured 6.6e-13: rocFFT vs numpy and the
    order of the f64 atomics)."""
    gp, op = _plan()
    uvw, sc, ec = _ref_inputs(3, seed=7)
    R = uvw.shape[0]
    img = wd.ref_image().astype(np.complex128)
    ref = op.degrid(img, *wd.REF_OFFSETS, C0, C0 / 100, uvw, sc, ec,
                    np.zeros((R, 3), np.complex128))
    v = _to(np.zeros((R, 3), np.complex128), device)
    gp.degrid(_to(img, device), *wd.REF_OFFSETS, C0, C0 / 100,
              _to(uvw, device), _to(sc, device), _to(ec, device), v)
    np.testing.assert_allclose(v.cpu().numpy(), ref, atol=1e-14, rtol=1e-13)
    rng = np.random.default_rng(8)
    vis = rng.normal(size=(R, 3)) + 1j * rng.normal(size=(R, 3))
    ref_img = op.grid(vis, uvw, sc, ec, C0, C0 / 100,
                      np.zeros((64, 64), np.complex128), *wd.REF_OFFSETS)
    out = _to(np.zeros((64, 64), np.complex128), device)
    gp.grid(_to(vis, device), _to(uvw, device), _to(sc, device),
            _to(ec, device), C0, C0 / 100, out, *wd.REF_OFFSETS)
    peak = np.abs(ref_img).max()
    assert peak > 100
    assert np.max(np.abs(out.cpu().numpy() - ref_img)) < 2e-12 * peak
