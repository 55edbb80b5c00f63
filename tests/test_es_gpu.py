"""GPU parity tests: HIP ES-FFT (de)gridder vs the CPU oracle.

Every test calls the product through its C ABI (ska_sdp_func ctypes wrapper
-> libska_sdp_func.so) on torch ROCm tensors and compares with oracle/ (the
CPU restatement of the reference, itself pinned by tests/test_oracle.py).

Tolerances (relative L2 over the whole output):
  f32: 1e-5  (north-star parity target; BASELINE.json)
  f64: 1e-12 (the reference's own double-precision adjointness threshold)
The taps are computed with the reference's arithmetic in both codes, so the
remaining differences are summation order and the f32 FFT.
"""
import numpy as np
import pytest

from es_data import make_case, reference_test_case, rel_l2
from oracle import es_oracle

pytestmark = pytest.mark.gpu

TOL = {False: 1e-5, True: 1e-12}


def _gpu(x, device):
    import torch

    return torch.from_numpy(np.ascontiguousarray(x)).to(device)


def _run_grid(device, uvw, freq, vis, wt, dirty0, px, eps, do_w):
    from ska_sdp_func.grid_data import GridderUvwEsFft

    g = [_gpu(a, device) for a in (uvw, freq, vis, wt, dirty0)]
    plan = GridderUvwEsFft(*g, px, px, eps, do_w)
    plan.grid_uvw_es_fft(*g)
    return g[4].cpu().numpy(), plan


def _run_degrid(device, uvw, freq, vis0, wt, dirty, px, eps, do_w):
    from ska_sdp_func.grid_data import GridderUvwEsFft

    g = [_gpu(a, device) for a in (uvw, freq, vis0, wt, dirty)]
    plan = GridderUvwEsFft(*g, px, px, eps, do_w)
    plan.ifft_grid_uvw_es(*g)
    return g[2].cpu().numpy(), g[4].cpu().numpy()


CASES = [
    # (dbl, do_w, rows, chan, N, eps)
    (False, False, 3000, 3, 256, 1e-5),
    (True, False, 3000, 3, 256, 1e-12),
    (False, True, 1500, 2, 256, 1e-5),
    (True, True, 1500, 2, 256, 1e-10),
    (False, False, 20000, 1, 840, 0.05),   # config-1 kernel (G=1024, W=4)
    # > 16 bucketing chunks of 8192 visibilities: every scan wave owns
    # several chunk slots, walked XCD by XCD (k_scan_columns)
    (False, False, 600000, 1, 256, 1e-5),
    (False, True, 150000, 4, 256, 1e-5),
    # 256 < entries per tile <= 1024: degrid pieces sorted by first-tap
    # sub-tile before the gather (k_sort_pieces)
    (False, False, 20000, 1, 256, 1e-5),
    (False, True, 8000, 2, 256, 1e-5),
    (False, False, 100000, 1, 840, 0.05),
    # 140000 rows x 64 channels: the chunk count is capped (kMaxChunks
    # 1024), chunks of ceil(140000 / 1024) = 137 rows, and the last three
    # chunks start past the last row (empty; k_bucket_fill once read past
    # the arrays for them)
    (False, False, 140000, 64, 256, 1e-5),
    (False, True, 140000, 64, 256, 1e-5),
    # f32 at eps 1e-7: W = 16, the 17-slot tap tables of the tile kernels
    (False, False, 3000, 3, 256, 1e-7),
    (False, True, 1500, 2, 256, 1e-7),
]


@pytest.mark.parametrize("dbl,do_w,rows,chan,n,eps", CASES)
def test_grid_matches_oracle(device, dbl, do_w, rows, chan, n, eps):
    uvw, freq, vis, wt, px = make_case(1, rows, chan, n, dbl=dbl,
                                       w_range=200.0)
    rdt = np.float64 if dbl else np.float32
    dirty0 = np.zeros((n, n), rdt)
    out, plan = _run_grid(device, uvw, freq, vis, wt, dirty0, px, eps, do_w)
    geo = es_oracle.geometry_for(uvw, freq, vis, dirty0, px, eps, do_w)
    assert plan.grid_size == geo["grid_size"]
    assert plan.support == geo["support"]
    assert plan.num_w_planes == geo["num_w_planes"]
    ref = es_oracle.grid_uvw_es_fft(geo, uvw, freq, vis, wt, dirty0)
    assert out.dtype == rdt
    assert rel_l2(out, ref) < TOL[dbl]


@pytest.mark.parametrize("dbl,do_w,rows,chan,n,eps", CASES)
def test_degrid_matches_oracle(device, dbl, do_w, rows, chan, n, eps):
    uvw, freq, vis, wt, px = make_case(2, rows, chan, n, dbl=dbl,
                                       w_range=200.0)
    rdt = np.float64 if dbl else np.float32
    rng = np.random.default_rng(3)
    dirty = rng.standard_normal((n, n)).astype(rdt)
    vis0 = np.zeros_like(vis)
    out_vis, out_dirty = _run_degrid(device, uvw, freq, vis0, wt, dirty, px,
                                     eps, do_w)
    geo = es_oracle.geometry_for(uvw, freq, vis, dirty, px, eps, do_w)
    ref_vis, ref_dirty = es_oracle.ifft_degrid_uvw_es(geo, uvw, freq, dirty)
    assert rel_l2(out_vis, ref_vis) < TOL[dbl]
    # the input image is grid-corrected in place (reference .cpp:789-825)
    assert rel_l2(out_dirty, ref_dirty) < (1e-6 if not dbl else 1e-14)


def test_grid_accumulates_and_corrects_input(device):
    """dirty_out = (dirty_in + S) * corr, reference .cpp:663-741."""
    n = 128
    uvw, freq, vis, wt, px = make_case(4, 500, 2, n)
    dirty0 = np.random.default_rng(5).standard_normal((n, n)).astype(np.float32)
    out, _ = _run_grid(device, uvw, freq, vis, wt, dirty0, px, 1e-5, False)
    geo = es_oracle.geometry_for(uvw, freq, vis, dirty0, px, 1e-5, False)
    ref = es_oracle.grid_uvw_es_fft(geo, uvw, freq, vis, wt, dirty0)
    assert rel_l2(out, ref) < 1e-5


def test_hot_tile_multi_piece(device):
    """> kPiece entries in one 64x64 tile: split work items + atomics."""
    n = 256
    uvw, freq, vis, wt, px = make_case(6, 12000, 1, n, frac=0.01)
    dirty0 = np.zeros((n, n), np.float32)
    out, _ = _run_grid(device, uvw, freq, vis, wt, dirty0, px, 1e-5, False)
    geo = es_oracle.geometry_for(uvw, freq, vis, dirty0, px, 1e-5, False)
    ref = es_oracle.grid_uvw_es_fft(geo, uvw, freq, vis, wt, dirty0)
    assert rel_l2(out, ref) < 1e-5
    vis0 = np.zeros_like(vis)
    d = np.random.default_rng(7).standard_normal((n, n)).astype(np.float32)
    out_vis, _ = _run_degrid(device, uvw, freq, vis0, wt, d, px, 1e-5, False)
    ref_vis, _ = es_oracle.ifft_degrid_uvw_es(geo, uvw, freq, d)
    assert rel_l2(out_vis, ref_vis) < 1e-5


def test_out_of_band_and_integer_positions(device):
    """Taps beyond the grid edge are dropped (kernels.cu:332-335); exact
    integer positions give W+1 taps per axis."""
    n = 128
    uvw, freq, vis, wt, px = make_case(8, 800, 2, n, frac=0.7)
    uvw[:10, :2] = 0.0                       # u = v = 0 exactly
    dirty0 = np.zeros((n, n), np.float32)
    out, _ = _run_grid(device, uvw, freq, vis, wt, dirty0, px, 1e-5, False)
    geo = es_oracle.geometry_for(uvw, freq, vis, dirty0, px, 1e-5, False)
    ref = es_oracle.grid_uvw_es_fft(geo, uvw, freq, vis, wt, dirty0)
    assert rel_l2(out, ref) < 1e-5


def test_odd_image_size(device):
    """Odd N: the last row/column is never written (reference quirk)."""
    n = 255
    uvw, freq, vis, wt, px = make_case(9, 700, 1, n, dbl=True)
    dirty0 = np.full((n, n), 3.0)
    out, _ = _run_grid(device, uvw, freq, vis, wt, dirty0, px, 1e-12, False)
    geo = es_oracle.geometry_for(uvw, freq, vis, dirty0, px, 1e-12, False)
    ref = es_oracle.grid_uvw_es_fft(geo, uvw, freq, vis, wt, dirty0)
    assert rel_l2(out, ref) < 1e-12
    assert np.all(out[-1, :] == 3.0) and np.all(out[:, -1] == 3.0)


def test_split_scatter_finish_equals_grid(device):
    import torch
    from ska_sdp_func.grid_data import GridderUvwEsFft

    n = 256
    uvw, freq, vis, wt, px = make_case(10, 4000, 2, n)
    g = [_gpu(a, device) for a in (uvw, freq, vis, wt)]
    d1 = torch.zeros((n, n), dtype=torch.float32, device=device)
    d2 = torch.zeros_like(d1)
    plan = GridderUvwEsFft(*g, d1, px, px, 1e-5, False)
    plan.grid_uvw_es_fft(*g, d1)
    G = plan.grid_size
    half = len(uvw) // 2
    grids = []
    for sl in (slice(0, half), slice(half, None)):
        gr = torch.empty((G, G), dtype=torch.complex64, device=device)
        plan.grid_scatter(g[0][sl].contiguous(), g[1], g[2][sl].contiguous(),
                          g[3][sl].contiguous(), gr)
        grids.append(gr)
    total = grids[0] + grids[1]
    plan.grid_finish(total, d2)
    assert rel_l2(d2.cpu().numpy(), d1.cpu().numpy()) < 1e-6


@pytest.mark.parametrize("do_single", [True, False])
@pytest.mark.parametrize("do_w", [False, True])
def test_reference_adjointness(device, do_single, do_w):
    """The reference's own test (test_gridder_uvw_es_fft.py:381-518):
    <dirty, grid(vis)> == Re<vis, degrid(dirty)> to 1e-5 (sp) / 1e-12 (dp).
    Its data is partly out of band, exercising the clamped-tap path."""
    import torch
    from ska_sdp_func.grid_data import GridderUvwEsFft

    uvw, freqs, test_vis, weight, test_dirty, px = reference_test_case(
        do_single)
    g_uvw, g_f, g_w = (_gpu(a, device) for a in (uvw, freqs, weight))
    g_tvis = _gpu(test_vis, device)
    g_tdirty = _gpu(test_dirty, device)
    vis_gpu = torch.zeros(test_vis.shape, dtype=g_tvis.dtype, device=device)
    dirty_gpu = torch.zeros(test_dirty.shape, dtype=g_tdirty.dtype,
                            device=device)
    plan = GridderUvwEsFft(g_uvw, g_f, g_tvis, g_w, dirty_gpu, px, px, 1e-5,
                           do_w)
    plan.grid_uvw_es_fft(g_uvw, g_f, g_tvis, g_w, dirty_gpu)
    adj1 = np.vdot(dirty_gpu.cpu().numpy(), test_dirty)
    plan.ifft_grid_uvw_es(g_uvw, g_f, vis_gpu, g_w, g_tdirty)
    adj2 = np.vdot(vis_gpu.cpu().numpy(), test_vis).real
    adj_error = np.abs(adj1 - adj2) / np.maximum(np.abs(adj1), np.abs(adj2))
    assert adj_error < (1e-5 if do_single else 1e-12)


def test_host_arrays_rejected(device):
    """No CPU fallback: host buffers fail like the reference GPU build."""
    from ska_sdp_func.grid_data import GridderUvwEsFft
    from ska_sdp_func.utility import CError

    n = 64
    uvw, freq, vis, wt, px = make_case(11, 10, 1, n)
    dirty = np.zeros((n, n), np.float32)
    plan = GridderUvwEsFft(_gpu(uvw, device), _gpu(freq, device),
                           _gpu(vis, device), _gpu(wt, device),
                           _gpu(dirty, device), px, px, 1e-5, False)
    with pytest.raises(CError, match="Memory location mismatch"):
        plan.grid_uvw_es_fft(_gpu(uvw, device), freq, _gpu(vis, device),
                             _gpu(wt, device), _gpu(dirty, device))
    with pytest.raises(CError, match="Memory location mismatch"):
        plan.grid_uvw_es_fft(uvw, freq, vis, wt, dirty)


def test_plan_parameters_match_reference_golden(device):
    import json
    import os

    from ska_sdp_func.grid_data import GridderUvwEsFft

    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "golden", "es_params.json")) as f:
        gold = json.load(f)["params"]
    for p in gold:
        if p["N"] not in (256, 1024) or p["eps"] < 1e-6 and not p["double"]:
            continue
        dbl = bool(p["double"])
        uvw, freq, vis, wt, px = make_case(0, 4, 1, p["N"], dbl=dbl)
        dirty = np.zeros((p["N"], p["N"]), np.float64 if dbl else np.float32)
        plan = GridderUvwEsFft(*[_gpu(a, device) for a in
                                 (uvw, freq, vis, wt, dirty)],
                               px, px, p["eps"], False)
        assert plan.grid_size == p["grid_size"]
        assert plan.support == p["support"]
        assert plan.beta == pytest.approx(p["beta"] * p["support"], rel=1e-15)


@pytest.mark.parametrize("rows", [1, 5, 70, 3000])
def test_scatter_grid_matches_oracle(device, rows):
    """uv grid after the tile scatter (before the FFT) vs the oracle's."""
    import torch
    from ska_sdp_func.grid_data import GridderUvwEsFft

    n = 256
    uvw, freq, vis, wt, px = make_case(12, rows, 2, n)
    dirty = torch.zeros((n, n), dtype=torch.float32, device=device)
    g = [_gpu(a, device) for a in (uvw, freq, vis, wt)]
    plan = GridderUvwEsFft(*g, dirty, px, px, 1e-5, False)
    G = plan.grid_size
    grid = torch.full((G, G), 7.0, dtype=torch.complex64, device=device)
    plan.grid_scatter(*g, grid)
    geo = es_oracle.geometry_for(uvw, freq, vis, np.zeros((n, n), np.float32),
                                 px, 1e-5, False)
    ref = es_oracle.scatter(geo, uvw, freq, vis, wt)
    out = grid.cpu().numpy()
    bad = np.argwhere(np.abs(out - ref) > 2e-6 * np.abs(ref).max())
    assert len(bad) == 0, (len(bad), bad[:5], out[tuple(bad[0])],
                           ref[tuple(bad[0])])


@pytest.mark.parametrize("dbl", [False, True])
def test_zero_rows(device, dbl):
    """No visibility rows: gridding returns the corrected input image and
    degridding corrects the image in place with nothing to write (the
    reference's loops run zero times); no kernel may be launched with an
    empty grid. The empty device arrays are views of allocated tensors:
    like the reference (sdp_mem.cpp:643-647), a NULL data pointer makes an
    array "not complex", which the argument checks reject."""
    import torch
    from ska_sdp_func.grid_data import GridderUvwEsFft

    n = 128
    uvw, freq, vis, wt, px = make_case(4, 500, 2, n, dbl=dbl)
    rdt = np.float64 if dbl else np.float32
    eps = 1e-12 if dbl else 1e-5
    dirty0 = np.random.default_rng(8).standard_normal((n, n)).astype(rdt)
    geo = es_oracle.geometry_for(uvw[:0], freq, vis[:0], dirty0, px, eps,
                                 False)
    g_uvw, g_vis, g_wt = (_gpu(a, device)[:0] for a in (uvw, vis, wt))
    g_freq = _gpu(freq, device)
    g_dirty = _gpu(dirty0, device)
    plan = GridderUvwEsFft(g_uvw, g_freq, g_vis, g_wt, g_dirty, px, px, eps,
                           False)
    plan.grid_uvw_es_fft(g_uvw, g_freq, g_vis, g_wt, g_dirty)
    ref = es_oracle.grid_uvw_es_fft(geo, uvw[:0], freq, vis[:0], wt[:0],
                                    dirty0)
    assert rel_l2(g_dirty.cpu().numpy(), ref) < TOL[dbl]
    g_dirty = _gpu(dirty0, device)
    plan.ifft_grid_uvw_es(g_uvw, g_freq, g_vis, g_wt, g_dirty)
    torch.cuda.synchronize()
    ref_vis, ref_dirty = es_oracle.ifft_degrid_uvw_es(geo, uvw[:0], freq,
                                                      dirty0)
    assert tuple(g_vis.shape) == ref_vis.shape == (0, 2)
    assert rel_l2(g_dirty.cpu().numpy(), ref_dirty) < (1e-6 if not dbl
                                                       else 1e-14)
