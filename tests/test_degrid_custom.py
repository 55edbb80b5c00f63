"""sdp_degrid_uvw_custom (csrc/grid_data/sdp_degrid_uvw_custom.hip)
against the CPU oracle (oracle/degrid_custom_oracle.py, a restatement of
sdp_degrid_uvw_custom.cpp).

The oracle is pinned by its plain-loop form (the reference's loop order)
and by a known answer: with uvw = 0 every visibility sits at the grid
centre with fractional offsets 0, so one-hot kernels pick one grid cell.
GPU results agree with the oracle to 1e-12 relative (per-lane sums and a
wave reduction instead of the reference's sequential order). The case
shape is the reference test's (test_degrid_uvw_custom.py: 512^2 grid,
4 w planes, kernels 8 / 4 wide, oversampling 16000, 5 channels).
"""
import numpy as np
import pytest

from oracle import degrid_custom_oracle as do

REF = dict(theta=0.1, wstep=250.0, f0=100e6, df=0.1e6)


def make_case(T=4, B=14, C=5, P=1, X=512, Z=4, K=8, KW=4, os_=16000,
              seed=2, spread=1.0, w_neg=0.0):
    rng = np.random.default_rng(seed)
    grid = rng.random((C, Z, X, X, P)) + 1j * rng.random((C, Z, X, X, P))
    uvw = spread * rng.random((T, B, 3))
    # w_neg > 0: odd baselines get w down to -w_neg metres, some below
    # -wstep, whose w-kernel rows fall outside the table (left unwritten).
    if w_neg > 0:
        uvw[:, 1::2, 2] = -w_neg * rng.random((T, B // 2))
    uv_kernel = rng.random((os_, K))
    w_kernel = rng.random((os_, KW))
    return grid, uvw, uv_kernel, w_kernel


def test_oracle_vectorised_matches_loops():
    # uvw spread so that some visibilities leave the grid (not written).
    grid, uvw, ku, kw = make_case(T=2, B=5, C=3, P=4, X=64, os_=64,
                                  spread=40000.0)
    a = np.full((2, 5, 3, 4), 9 + 9j)
    b = a.copy()
    args = (grid, uvw, ku, kw, 0.01, 250.0, 100e6, 0.1e6)
    do.degrid(*args, False, a)
    do.degrid_loops(*args, False, b)
    assert np.count_nonzero(a == 9 + 9j) > 0          # some off the grid
    np.testing.assert_allclose(a, b, rtol=1e-13)
    grid, uvw, ku, kw = make_case(T=2, B=6, C=3, P=1, X=64, os_=64,
                                  w_neg=3000.0, seed=5)
    a = np.full((2, 6, 3, 1), 9 + 9j)
    b = a.copy()
    args = (grid, uvw, ku, kw, 0.01, 250.0, 100e6, 0.1e6)
    do.degrid(*args, False, a)
    do.degrid_loops(*args, False, b)
    assert np.count_nonzero(a[:, 1::2] == 9 + 9j) > 0   # w rows off table
    np.testing.assert_allclose(a, b, rtol=1e-13)
    do.degrid(*args, True, a)
    do.degrid_loops(*args, True, b)
    np.testing.assert_allclose(a, b, rtol=1e-13)


def test_oracle_known_answer():
    grid, _, _, _ = make_case(T=1, B=2, C=2, P=1, X=32, os_=16)
    uvw = np.zeros((1, 2, 3))
    ku = np.zeros((16, 8))
    ku[:, 3] = 1.0
    kw = np.zeros((16, 4))
    kw[:, 2] = 1.0
    vis = np.zeros((1, 2, 2, 1), complex)
    do.degrid(grid, uvw, ku, kw, 0.1, 250.0, 100e6, 1e6, False, vis)
    for c in range(2):
        assert vis[0, 0, c, 0] == grid[c, 2, 16 + 3 - 4, 16 + 3 - 4, 0]


def test_library_exports_degrid_custom():
    from ska_sdp_func.utility import Lib
    assert hasattr(Lib.handle(), "sdp_degrid_uvw_custom")


@pytest.mark.gpu
@pytest.mark.parametrize("on_device", [False, True])
@pytest.mark.parametrize("P,conj", [(1, False), (4, True)])
def test_gpu_matches_oracle(device, on_device, P, conj):
    from ska_sdp_func.grid_data import degrid_uvw_custom
    for kw_args in (dict(P=P), dict(P=P, X=128, os_=64, spread=4000.0,
                                    T=8, B=40),
                    dict(P=P, X=128, os_=64, spread=4000.0, T=8, B=40,
                         w_neg=2500.0)):
        grid, uvw, ku, kw = make_case(**kw_args)
        shape = uvw.shape[:2] + (grid.shape[0], P)
        ref = np.full(shape, 5 - 5j)
        do.degrid(grid, uvw, ku, kw, REF["theta"], REF["wstep"], REF["f0"],
                  REF["df"], conj, ref)
        out = np.full(shape, 5 - 5j)
        arrays = [grid, uvw, ku, kw]
        if on_device:
            import torch
            arrays = [torch.from_numpy(a).to(device) for a in arrays]
            o = torch.from_numpy(out).to(device)
        else:
            o = out
        degrid_uvw_custom(*arrays, REF["theta"], REF["wstep"], REF["f0"],
                          REF["df"], conj, o)
        if on_device:
            out = o.cpu().numpy()
        np.testing.assert_allclose(out, ref, rtol=1e-12)


@pytest.mark.gpu
def test_gpu_argument_errors(device):
    from ska_sdp_func.grid_data import degrid_uvw_custom
    from ska_sdp_func.utility import CError
    grid, uvw, ku, kw = make_case(T=1, B=2, C=1, X=32, os_=16)
    vis = np.zeros((1, 2, 1, 1), complex)
    a = (0.1, 250.0, 100e6, 0.1e6, False)
    with pytest.raises(CError, match="Unsupported data type"):
        degrid_uvw_custom(grid.astype(np.complex64), uvw, ku, kw, *a, vis)
    with pytest.raises(CError, match="Invalid function argument"):
        degrid_uvw_custom(grid, uvw, ku, kw, *a,
                          np.zeros((1, 2, 1, 2), complex))
    with pytest.raises(CError, match="Unsupported data type"):
        degrid_uvw_custom(grid, uvw, ku, kw, *a, np.zeros((1, 2, 1, 1)))
