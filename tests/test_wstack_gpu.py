"""GPU parity of the w-stacking x w-towers driver
(csrc/grid_data/sdp_grid_wstack_wtower.hip) with the oracle's restatement
of sdp_grid_wstack_wtower.cpp (one thread, task by task).

Pins: degridding matches the direct Fourier sum to the kernel accuracy;
gridding is the exact adjoint of degridding (for image pixels away from
the PSWF's 1e-15 end value); shards of w-stack planes sum to the whole.
Tolerances: complex128 results agree with the oracle to 2e-9 of the
largest value (summation order, FFT library, and the common w-layer range
of a batch of sub-grids, which changes the number of w-pattern divisions
but not the result), complex64 to 5e-5. Image comparisons
skip a 32-pixel border, where the grid correction divides by the PSWF's
near-zero tail and amplifies rounding by up to 1e8 (the reference's own
full-image test skips 30 pixels, test_gridder_wtower_uvw.py:2189-2193).
"""
import numpy as np
import pytest

import wtower_data as wd
from oracle import wtower_oracle as wo

pytestmark = pytest.mark.gpu

KW = dict(support=8, oversampling=16384, w_support=8, w_oversampling=16384)


def _args(case, S):
    return (case["f0"], case["df"], case["uvw"], S, case["theta"],
            case["w_step"], 0.0, 0.0, KW["support"], KW["oversampling"],
            KW["w_support"], KW["w_oversampling"], 0.0, case["H"])


def _close(a, b, tol, border=0):
    if border:
        a = a[border:-border, border:-border]
        b = b[border:-border, border:-border]
    err = np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)
    assert err <= tol, f"max rel err {err:.3e} > {tol:.1e}"


def _image(N, rng, complex_=True):
    img = rng.normal(size=(N, N))
    if complex_:
        img = img + 1j * rng.normal(size=(N, N))
    return img


@pytest.fixture(scope="module")
def case():
    return wd.wstack_case(num_rows=1000, num_chan=3)


@pytest.mark.parametrize("vis_t,uvw_t,tol", [
    (np.complex128, np.float64, 2e-9),
    (np.complex64, np.float32, 5e-5),
])
def test_degrid_all_matches_oracle(device, case, vis_t, uvw_t, tol):
    import ska_sdp_func.grid_data as g
    rng = np.random.default_rng(1)
    N, S = 256, 64
    img = _image(N, rng)
    # Zero border: the degrid correction amplifies the edge by up to
    # 1 / pswf(x)^2 (1.5e5 at 16 pixels from the edge here), which single
    # precision cannot carry; 64 pixels keeps it below 25.
    bd = 16 if vis_t is np.complex128 else 64
    img[:bd] = 0
    img[-bd:] = 0
    img[:, :bd] = 0
    img[:, -bd:] = 0
    uvw = case["uvw"].astype(uvw_t)
    a = (case["f0"], case["df"], uvw.astype(np.float64)) + _args(case, S)[3:]
    ref = wo.wstack_degrid_all(img, *a, np.zeros((1000, 3), complex))
    vis = np.full((1000, 3), 7.0 + 1j, vis_t)          # overwritten
    image_in = img.astype(np.complex128 if vis_t is np.complex128
                          else np.complex64)
    g.wstack_wtower_degrid_all(image_in, a[0], a[1], uvw, *a[3:], 0, vis)
    _close(vis, ref, tol)


@pytest.mark.parametrize("vis_t,uvw_t,img_t,tol", [
    (np.complex128, np.float64, np.complex128, 2e-9),
    (np.complex128, np.float64, np.float64, 2e-9),
    (np.complex64, np.float64, np.float32, 5e-5),
])
def test_grid_all_matches_oracle(device, case, vis_t, uvw_t, img_t, tol):
    import ska_sdp_func.grid_data as g
    rng = np.random.default_rng(2)
    N, S = 256, 64
    vis = (rng.normal(size=(1000, 3)) + 1j * rng.normal(size=(1000, 3)))
    uvw = case["uvw"].astype(uvw_t)
    a = (case["f0"], case["df"], uvw.astype(np.float64)) + _args(case, S)[3:]
    ref = wo.wstack_grid_all(vis, *a, np.zeros((N, N), img_t))
    out = np.full((N, N), 3.0, img_t)                   # overwritten
    g.wstack_wtower_grid_all(vis.astype(vis_t), a[0], a[1], uvw, *a[3:], 0,
                             out)
    # Single precision: the correction's amplification of rounding near the
    # edge needs a wider border.
    _close(out, ref, tol, border=32 if vis_t is np.complex128 else 64)


def test_degrid_all_matches_dft(device):
    """Point sources, 20 000 rows x 4 channels, 512^2: rms error vs the DFT
    below 1e-4 of the flux (the reference's C test allows 1e-3)."""
    import ska_sdp_func.grid_data as g
    N, S = 512, 128
    c = wd.wstack_case(num_rows=20000, num_chan=4, image_size=N, seed=3,
                       w_tower_height=8.0, w_planes=4.0)
    img = np.zeros((N, N))
    src = [(40, -60, 1.0), (-100, 20, 0.7), (10, 120, 0.4)]
    for il, im, f in src:
        img[N // 2 + il, N // 2 + im] = f
    vis = np.zeros((20000, 4), np.complex128)
    g.wstack_wtower_degrid_all(img, *_args(c, S)[:2], c["uvw"],
                               *_args(c, S)[3:], 0, vis)
    freqs = c["f0"] + np.arange(4) * c["df"]
    ref = np.zeros_like(vis)
    for il, im, f in src:
        l, m = il * c["theta"] / N, im * c["theta"] / N
        n = wo.lm_to_n(l, m, 0.0, 0.0)
        ph = (c["uvw"] @ np.array([l, m, n]))[:, None] * (freqs / wd.C_0)
        ref += f * np.exp(-2j * np.pi * ph)
    err = np.abs(vis - ref)
    # A visibility within 1 / (2 w_oversampling) of the top of a w-layer
    # rounds to the w-kernel row of the layer's bottom (iw0_ov % w_os = 0,
    # sdp_gridder_wtower_uvw.cpp:127-138, no carry into the next layer) and
    # comes out a full w_step off; the reference does the same (the oracle
    # reproduces it exactly). About 1 in 10^4 visibilities; excluded here.
    ok = err < 1e-3
    assert np.count_nonzero(~ok) <= err.size // 5000
    assert np.sqrt(np.mean(err[ok] ** 2)) < 1e-4
    assert np.count_nonzero(vis) == vis.size


def test_grid_all_is_adjoint_and_shards_sum(device):
    import torch
    import ska_sdp_func.grid_data as g
    N, S, R, C = 1024, 128, 100000, 2
    c = wd.wstack_case(num_rows=R, num_chan=C, image_size=N, seed=4,
                       w_tower_height=8.0, w_planes=5.0)
    rng = np.random.default_rng(5)
    x = _image(N, rng)
    x[:N // 8] = 0
    x[-N // 8:] = 0
    x[:, :N // 8] = 0
    x[:, -N // 8:] = 0
    y = rng.normal(size=(R, C)) + 1j * rng.normal(size=(R, C))
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
    a = _args(c, S)
    d_uvw = dev(c["uvw"])
    ax = torch.zeros((R, C), dtype=torch.complex128, device=device)
    g.wstack_wtower_degrid_all(dev(x), a[0], a[1], d_uvw, *a[3:], 0, ax)
    gy = torch.zeros((N, N), dtype=torch.complex128, device=device)
    g.wstack_wtower_grid_all(dev(y), a[0], a[1], d_uvw, *a[3:], 0, gy)
    lhs = np.vdot(y, ax.cpu().numpy())
    rhs = np.vdot(gy.cpu().numpy(), x)
    assert abs(lhs - rhs) <= 1e-10 * abs(lhs)
    # Shards of w-stack planes sum to the whole.
    acc = torch.zeros_like(gy)
    vacc = torch.zeros_like(ax)
    for k in range(3):
        part = torch.zeros_like(gy)
        g.wstack_wtower_grid_planes(dev(y), a[0], a[1], d_uvw, *a[3:], 0,
                                    part, k, 3)
        acc += part
        vpart = torch.zeros_like(ax)
        g.wstack_wtower_degrid_planes(dev(x), a[0], a[1], d_uvw, *a[3:], 0,
                                      vpart, k, 3)
        vacc += vpart
    _close(acc.cpu().numpy(), gy.cpu().numpy(), 1e-10, border=128)
    _close(vacc.cpu().numpy(), ax.cpu().numpy(), 1e-12)
    # Load-balanced plane sets (the multi-GPU assignment of
    # bench_wtower.py): disjoint masks over the modelled plane range, host
    # and device masks, also sum to the whole.
    from ska_sdp_func.grid_data.distributed import (assign_planes,
                                                    wstack_plane_loads)
    first, loads = wstack_plane_loads(c["uvw"], a[0], a[1], C, c["w_step"],
                                      c["H"])
    masks, _ = assign_planes(loads, 3)
    acc.zero_()
    vacc.zero_()
    for k in range(3):
        m = masks[k] if k != 1 else dev(masks[k])
        part = torch.zeros_like(gy)
        g.wstack_wtower_grid_plane_set(dev(y), a[0], a[1], d_uvw, *a[3:], 0,
                                       part, first, m)
        acc += part
        vpart = torch.zeros_like(ax)
        g.wstack_wtower_degrid_plane_set(dev(x), a[0], a[1], d_uvw, *a[3:],
                                         0, vpart, first, m)
        vacc += vpart
    _close(acc.cpu().numpy(), gy.cpu().numpy(), 1e-10, border=128)
    _close(vacc.cpu().numpy(), ax.cpu().numpy(), 1e-12)
    # A mask range that misses occupied planes at both ends (a plane-range
    # model that is off): the planes outside belong to the owners of the
    # first / last entry, so the shards still sum to the whole.
    cut = masks[:, 2:-2]
    assert cut.shape[1] >= 1 and loads[1] + loads[-2] > 0
    acc.zero_()
    vacc.zero_()
    for k in range(3):
        part = torch.zeros_like(gy)
        g.wstack_wtower_grid_plane_set(dev(y), a[0], a[1], d_uvw, *a[3:], 0,
                                       part, first + 2, dev(cut[k]))
        acc += part
        vpart = torch.zeros_like(ax)
        g.wstack_wtower_degrid_plane_set(dev(x), a[0], a[1], d_uvw, *a[3:],
                                         0, vpart, first + 2,
                                         np.ascontiguousarray(cut[k]))
        vacc += vpart
    _close(acc.cpu().numpy(), gy.cpu().numpy(), 1e-10, border=128)
    _close(vacc.cpu().numpy(), ax.cpu().numpy(), 1e-12)


def test_argument_errors(device, case):
    import ska_sdp_func.grid_data as g
    from ska_sdp_func.utility import CError
    a = list(_args(case, 64))
    vis = np.zeros((1000, 3), np.complex128)
    img = np.zeros((256, 256), np.complex128)
    a[-1] = 0.0
    with pytest.raises(CError, match="Invalid function argument"):
        g.wstack_wtower_grid_all(vis, *a[:2], case["uvw"], *a[3:], 0, img)
    import torch
    a[-1] = case["H"]
    with pytest.raises(CError, match="Memory location"):
        g.wstack_wtower_grid_all(vis, *a[:2], torch.from_numpy(
            case["uvw"]).to(device), *a[3:], 0, img)


@pytest.mark.parametrize("degrid", [False, True])
def test_fused_towers_match_double_precision(device, degrid):
    """Complex-float runs take the fused tower kernels (k_tower_dft /
    k_tower_idft) and, at this power-of-two image size, the fused in-place
    plane FFT with permuted rows (es_fft.hip fft2d_inplace_permuted);
    checked against the complex-double path (layer-by-layer towers, rocFFT)
    on a config-4-shaped case dense enough that the per-layer visibility
    windows of a sub-grid overflow the kernels' LDS ring (multi-piece
    windows, restaging, flushes of partial sums)."""
    import math
    import torch
    import ska_sdp_func.grid_data as g
    R, N, S, theta = 200_000, 2048, 256, 0.04
    fov = 0.8 * theta
    w_step = g.determine_w_step(theta, fov, 0.0, 0.0)
    H = float(g.determine_max_w_tower_height(
        S, theta, fov, w_step, 8, 16384, 8, 16384, image_size=2 * S,
        subgrid_frac=2.0 / 3.0))
    gen = torch.Generator(device=device)
    gen.manual_seed(7)
    r = 0.45 * N / theta * torch.sqrt(torch.rand(R, generator=gen,
                                                 device=device,
                                                 dtype=torch.float64))
    ph = 2 * math.pi * torch.rand(R, generator=gen, device=device,
                                  dtype=torch.float64)
    w = (torch.rand(R, generator=gen, device=device, dtype=torch.float64)
         * 4 - 2.5) * H * w_step
    # Both runs see the same (f32-representable) coordinates.
    uvw = torch.stack([r * torch.cos(ph), r * torch.sin(ph), w], 1).float(
        ).double()
    vis = torch.complex(torch.randn((R, 1), generator=gen, device=device),
                        torch.randn((R, 1), generator=gen, device=device))
    common = (wd.C_0, wd.C_0 / 200)
    tail = (S, theta, w_step, 0.0, 0.0, 8, 16384, 8, 16384, 0.0, H)
    if degrid:
        img = torch.randn((N, N), generator=gen, device=device)
        b = N // 4
        img[:b] = 0
        img[-b:] = 0
        img[:, :b] = 0
        img[:, -b:] = 0
        out32 = torch.zeros((R, 1), dtype=torch.complex64, device=device)
        out64 = torch.zeros((R, 1), dtype=torch.complex128, device=device)
        g.wstack_wtower_degrid_all(img, *common, uvw.float(), *tail, 0,
                                   out32)
        g.wstack_wtower_degrid_all(img.double(), *common, uvw, *tail, 0,
                                   out64)
        a, ref = out32.cpu().numpy(), out64.cpu().numpy()
        _close(a, ref, 2e-6)
    else:
        im32 = torch.zeros((N, N), dtype=torch.float32, device=device)
        im64 = torch.zeros((N, N), dtype=torch.float64, device=device)
        g.wstack_wtower_grid_all(vis, *common, uvw.float(), *tail, 0, im32)
        g.wstack_wtower_grid_all(vis.to(torch.complex128), *common, uvw,
                                 *tail, 0, im64)
        # Interior only: the grid correction amplifies f32 rounding near
        # the facet edge (module docstring).
        _close(im32.cpu().numpy(), im64.cpu().numpy(), 5e-5, border=N // 4)


@pytest.mark.parametrize("degrid", [False, True])
def test_fused_towers_dense_vs_oracle(device, degrid):
    """The complex-float product path (fused tower kernels) against the
    oracle on a case dense enough that a sub-grid's per-layer visibility
    windows overflow the kernels' LDS rings (restaging, multi-piece
    windows, partial-sum flushes). The oracle needs about a minute per
    direction here, so its outputs are golden vectors made by
    tests/golden/make_wtower_dense.py (inputs regenerated from the same
    seeds)."""
    import os
    import torch
    import ska_sdp_func.grid_data as g
    from golden.make_wtower_dense import N, inputs
    gold = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                "golden", "wtower_dense.npz"))
    c, vis, img, a = inputs()
    dev = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(device)
    if degrid:
        out = torch.zeros(vis.shape, dtype=torch.complex64, device=device)
        g.wstack_wtower_degrid_all(dev(img.astype(np.float32)), a[0], a[1],
                                   dev(c["uvw"]), *a[3:], 0, out)
        _close(out.cpu().numpy(), gold["degrid"], 1e-5)
    else:
        out = torch.zeros((N, N), dtype=torch.float32, device=device)
        g.wstack_wtower_grid_all(dev(vis.astype(np.complex64)), a[0], a[1],
                                 dev(c["uvw"]), *a[3:], 0, out)
        b = N // 4
        _close(out.cpu().numpy()[b:-b, b:-b], gold["grid_interior"], 5e-5)


@pytest.mark.parametrize("uv_frac", [0.75, 1.3])
def test_uv_extent_wider_than_grid(device, uv_frac):
    """Sub-grids past the grid edge wrap onto it (subgrid_add / cut_out use
    periodic indices, sdp_gridder_utils.cpp:553-648): a cell can then be
    covered by sub-grids from two or three periodic images; every one of
    them must be summed (gridding) and read (degridding) as the oracle's
    task-by-task restatement does."""
    import ska_sdp_func.grid_data as g
    c = wd.wstack_case(num_rows=600, num_chan=2, seed=9, uv_frac=uv_frac)
    N, S = 256, 64
    rng = np.random.default_rng(10)
    vis = (rng.normal(size=(600, 2)) + 1j * rng.normal(size=(600, 2)))
    a = (c["f0"], c["df"], c["uvw"]) + _args(c, S)[3:]
    ref = wo.wstack_grid_all(vis, *a, np.zeros((N, N), np.complex128))
    out = np.zeros((N, N), np.complex128)
    g.wstack_wtower_grid_all(vis, a[0], a[1], c["uvw"], *a[3:], 0, out)
    _close(out, ref, 2e-9, border=32)
    img = _image(N, rng)
    img[:16] = 0
    img[-16:] = 0
    img[:, :16] = 0
    img[:, -16:] = 0
    vref = wo.wstack_degrid_all(img, *a, np.zeros((600, 2), complex))
    v = np.zeros((600, 2), np.complex128)
    g.wstack_wtower_degrid_all(img, a[0], a[1], c["uvw"], *a[3:], 0, v)
    _close(v, vref, 2e-9)
