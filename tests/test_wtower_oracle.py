"""W-towers oracle checks (CPU).

The oracle (oracle/wtower_oracle.py) restates sdp_gridder_wtower_uvw.cpp
and its helpers. The reference itself could not be run here (DESIGN.md,
"Denied"), so the oracle is pinned by physics and by exact identities:
  * degridding a corrected sub-grid image reproduces the direct Fourier sum
    (to the accuracy the reference's PSWF-window design allows),
  * gridding followed by grid correction reproduces the inverse DFT,
  * gridding is the exact adjoint of degridding,
  * the vectorised channel clamp equals the scalar restatement.
The host-side table generators of the library (PSWF kernels, w-pattern,
w step, worst-case image) run without a GPU and are compared here too.
"""
import math

import numpy as np
import pytest

from oracle import wtower_oracle as wo
import wtower_data as wd

C0 = wd.C_0


def _rand_uvw(rng, n, uv, w):
    uvw = np.zeros((n, 3))
    uvw[:, :2] = rng.uniform(-uv, uv, (n, 2))
    uvw[:, 2] = rng.uniform(-w, w, n)
    return uvw


@pytest.mark.parametrize("shear", [(0.0, 0.0), (0.2, 0.1)])
@pytest.mark.parametrize("w_max", [0.0, 30000.0])
def test_oracle_degrid_matches_dft(shear, w_max):
    S = N = 64
    theta = 0.01
    p = wo.WtowerPlan(N, S, theta, 2000.0, *shear, 10, 16384, 10, 16384)
    rng = np.random.default_rng(1)
    R = 200
    uvw = _rand_uvw(rng, R, 2500.0, w_max)
    img = np.zeros((S, S), complex)
    for il, im, f in [(5, -7, 1.0), (-10, 3, 0.5), (0, 0, 0.25)]:
        img[S // 2 + il, S // 2 + im] = f
    corr = p.degrid_correct(img.copy(), 0, 0)
    sc = np.zeros(R, np.int32)
    ec = np.ones(R, np.int32)
    vis = p.degrid(corr, 0, 0, 0, C0, C0 / 100, uvw, sc, ec,
                   np.zeros((R, 1), complex))
    ref = wo.dft_subgrid_vis(img, theta, *shear, uvw)
    # Accuracy floor of the reference design: the uv kernel is the DFT of
    # the PSWF window sampled at `support` points (utils.cpp:385-427).
    assert np.abs(vis[:, 0] - ref).max() < 2e-4
    if w_max:
        assert p.num_w_planes[0] > 10


def test_oracle_grid_matches_idft():
    S = N = 64
    theta = 0.01
    shear = (0.2, 0.1)
    p = wo.WtowerPlan(N, S, theta, 2000.0, *shear, 10, 16384, 10, 16384)
    rng = np.random.default_rng(3)
    R = 150
    uvw = _rand_uvw(rng, R, 2500.0, 20000.0)
    vis = rng.normal(size=(R, 1)) + 1j * rng.normal(size=(R, 1))
    sub = np.zeros((S, S), complex)
    p.grid(vis, uvw, np.zeros(R, np.int32), np.ones(R, np.int32), C0,
           C0 / 100, sub, 0, 0, 0)
    p.grid_correct(sub, 0, 0)
    l = (np.arange(S) - S // 2) * theta / S
    L, M = np.meshgrid(l, l, indexing="ij")
    n = wo.lm_to_n(L, M, *shear)
    ph = (uvw[:, 0, None] * L.ravel() + uvw[:, 1, None] * M.ravel()
          + uvw[:, 2, None] * n.ravel())
    ref = (np.exp(2j * np.pi * ph).T @ vis[:, 0]).reshape(S, S)
    c = slice(S // 4, 3 * S // 4)
    assert np.abs(sub - ref)[c, c].max() < 1e-4 * np.abs(ref).max()


def test_oracle_grid_is_adjoint_of_degrid():
    S, N, theta = 64, 256, 0.01
    p = wo.WtowerPlan(N, S, theta, 2000.0, 0.2, 0.1, 10, 16384, 10, 16384)
    rng = np.random.default_rng(2)
    R, C = 300, 3
    uvw = _rand_uvw(rng, R, 2000.0, 20000.0)
    sc = rng.integers(0, 2, R).astype(np.int32)
    ec = np.full(R, C, np.int32)
    x = rng.normal(size=(S, S)) + 1j * rng.normal(size=(S, S))
    y = (rng.normal(size=(R, C)) + 1j * rng.normal(size=(R, C)))
    y *= np.arange(C)[None, :] >= sc[:, None]
    ax = p.degrid(x, 3, -2, 1, C0, C0 / 50, uvw, sc, ec,
                  np.zeros((R, C), complex))
    gy = np.zeros((S, S), complex)
    p.grid(y, uvw, sc, ec, C0, C0 / 50, gy, 3, -2, 1)
    lhs, rhs = np.vdot(y, ax), np.vdot(gy, x)
    assert abs(lhs - rhs) <= 1e-12 * abs(lhs)
    assert p.num_w_planes[0] == p.num_w_planes[1] > 10


def test_oracle_reference_config_selects_rows():
    """The test sub-grid sees most of the synthetic Y-array's rows on many
    w-planes."""
    cfg = wd.REF_CFG
    p = wo.WtowerPlan(**cfg)
    uvw = wd.generate_uvw()
    R = uvw.shape[0]
    sc = np.zeros(R, np.int32)
    ec = np.full(R, 2, np.int32)
    vis = p.degrid(wd.ref_image().astype(complex), *wd.REF_OFFSETS, C0,
                   C0 / 100, uvw, sc, ec, np.zeros((R, 2), complex))
    hit = np.count_nonzero(vis)
    assert vis.size // 2 < hit < vis.size
    assert p.num_w_planes[0] > 100


def test_clamp_vec_matches_scalar():
    rng = np.random.default_rng(7)
    n = 2000
    u = rng.normal(0, 3000, n)
    u[::17] = 0.0
    u[::29] = 1e-9
    s = rng.integers(0, 10, n)
    e = s + rng.integers(-2, 40, n)
    for lo, hi in [(-500.0, 700.0), (0.0, 280.0), (-1e4, -2e3)]:
        vs, ve = wo.clamp_channels_vec(u, C0, C0 / 100, s, e, lo, hi)
        for i in range(n):
            assert (vs[i], ve[i]) == wo.clamp_channels(
                u[i], C0, C0 / 100, int(s[i]), int(e[i]), lo, hi)


def test_clamp_selects_exactly_the_range():
    """clamp_channels keeps exactly the channels with min <= u_c < max."""
    rng = np.random.default_rng(8)
    f0, df = 1.0e8, 1.0e6
    for _ in range(500):
        u = rng.normal(0, 5000)
        lo = rng.uniform(-3000, 3000)
        hi = lo + rng.uniform(1, 500)
        s, e = wo.clamp_channels(u, f0, df, 0, 64, lo, hi)
        inside = [c for c in range(64)
                  if lo <= (f0 + c * df) * u / C0 < hi]
        if inside:
            # Rounding at the interval ends may move one boundary channel.
            assert abs(s - inside[0]) <= 1 and abs(e - (inside[-1] + 1)) <= 1
        else:
            assert e - s <= 1


# -- library host-side generators (no GPU involved) -------------------------

def _lib():
    pytest.importorskip("ska_sdp_func")
    import ska_sdp_func.grid_data as g
    return g


@pytest.mark.parametrize("support", [6, 8, 10])
def test_make_pswf_kernel_matches_oracle(support):
    g = _lib()
    os_ = 64
    k = np.zeros((os_ + 1, support))
    g.make_pswf_kernel(support, k)
    ref = wo.make_pswf_kernel(support, os_)
    np.testing.assert_allclose(k, ref, rtol=1e-10, atol=1e-14)


def test_make_kernel_matches_oracle():
    g = _lib()
    rng = np.random.default_rng(123)
    window = rng.random(10)
    k = np.zeros((129, 10))
    g.make_kernel(window, k)
    np.testing.assert_allclose(k, wo.make_kernel(window, 128), rtol=1e-12,
                               atol=1e-15)


def test_make_w_pattern_matches_oracle():
    g = _lib()
    cfg = wd.REF_CFG
    w = np.zeros((64, 64), np.complex128)
    g.make_w_pattern(64, cfg["theta"], 0.2, 0.1, cfg["w_step"], w)
    ref = wo.make_w_pattern(64, cfg["theta"], 0.2, 0.1, cfg["w_step"])
    np.testing.assert_allclose(w, ref, rtol=1e-14, atol=1e-15)


def test_determine_w_step_matches_oracle():
    g = _lib()
    for theta, fov, hu, hv in [(0.01, 0.008, 0.0, 0.0), (0.1, 0.05, 0.2, 0.1)]:
        assert math.isclose(g.determine_w_step(theta, fov, hu, hv),
                            wo.determine_w_step(theta, fov, hu, hv),
                            rel_tol=1e-14)


def test_worst_case_image():
    import ctypes
    from ska_sdp_func.utility import Lib, Mem
    _lib()
    Lib.wrap_func("sdp_gridder_worst_case_image", restype=None,
                  argtypes=[ctypes.c_double, ctypes.c_double,
                            Mem.handle_type()], check_errcode=True)
    img = np.zeros((128, 128), np.complex128)
    Lib.sdp_gridder_worst_case_image(0.01, 0.008, Mem(img))
    # fov_edge = int(128 / 0.01 * 0.008 / 2) = 51 (not a divisor of 128).
    nz = {tuple(ix): img[tuple(ix)].real for ix in np.argwhere(img != 0)}
    assert nz == {(115, 115): 0.3, (13, 13): 0.2, (115, 12): 0.3,
                  (12, 115): 0.2}


def test_python_api_errors_without_gpu():
    """Argument checks that happen before any device work."""
    g = _lib()
    from ska_sdp_func.utility import CError
    with pytest.raises(CError, match="Invalid function argument"):
        g.GridderWtowerUVW(256, 63, 0.01, 100.0, 0, 0, 10, 16384, 10, 16384)
    gp = g.GridderWtowerUVW(**wd.REF_CFG)
    assert (gp.image_size, gp.subgrid_size, gp.support, gp.oversampling,
            gp.w_support, gp.w_oversampling) == (256, 64, 10, 16384, 10,
                                                 16384)
    assert (gp.theta, gp.w_step, gp.shear_u, gp.shear_v) == (0.0008, 280.0,
                                                             0.2, 0.1)
    vis = np.zeros((10, 3), np.complex128)
    with pytest.raises(RuntimeError, match="Inconsistent channel dimensions"):
        gp.grid_subgrid(vis, np.zeros((10, 3)), np.zeros(10, np.int32),
                        np.ones(10, np.int32), 2, C0, C0 / 100,
                        np.zeros((64, 64), np.complex128), (0, 0, 0))


def test_dense_golden_vectors_match_their_case():
    """tests/golden/wtower_dense.npz (made by make_wtower_dense.py from the
    oracle) fits the case the GPU test regenerates: shapes, finite values,
    every visibility degridded, and a spot check of one visibility against
    the oracle's single-row degridding."""
    import os
    from golden.make_wtower_dense import N, inputs
    gold = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                "golden", "wtower_dense.npz"))
    c, vis, img, a = inputs()
    assert gold["grid_interior"].shape == (N // 2, N // 2)
    assert gold["degrid"].shape == vis.shape
    assert np.all(np.isfinite(gold["grid_interior"]))
    assert np.count_nonzero(gold["degrid"]) == vis.size
    # The visibilities are independent: degridding the first 4 rows alone
    # gives the same values (cheap: few sub-grids).
    part = wo.wstack_degrid_all(img, a[0], a[1], c["uvw"][:4], *a[3:],
                                np.zeros((4, 1), complex))
    np.testing.assert_allclose(part, gold["degrid"][:4], rtol=1e-5,
                               atol=1e-6 * np.abs(gold["degrid"]).max())
