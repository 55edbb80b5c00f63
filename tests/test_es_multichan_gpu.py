"""GPU parity of multi-channel 2-D gridding (f32, 8 to 64 channels per row)
at the edges of the bucketing: channel counts that are not a multiple of
anything convenient, descending and shuffled frequencies (the channels of
a row then jump between tiles), channels whose taps leave the grid,
exact-integer positions (W + 1 taps), W = 16 and W = 4 plans, tiles with
more entries than one work item (pieces combined by atomics), the split
scatter API and row batches. (Written for the round-5 channel-run
bucketing, which was measured and removed)
Reference: the oracle (oracle/es_oracle.c, a restatement of
sdp_gridder_uvw_es_fft_kernels.cu:277-422), relative L2 <= 1e-5 (f32,
BASELINE north star).
"""
import numpy as np
import pytest

from es_data import make_case, rel_l2
from oracle import es_oracle

pytestmark = pytest.mark.gpu


def _gpu(x, device):
    import torch

    return torch.from_numpy(np.ascontiguousarray(x)).to(device)


def _order(freq, mode, seed):
    if mode == "descending":
        return freq[::-1].copy()
    if mode == "shuffled":
        return np.random.default_rng(seed).permutation(freq)
    return freq


def _grid(device, uvw, freq, vis, wt, n, px, eps, cap=None):
    from ska_sdp_func.grid_data import GridderUvwEsFft

    dirty0 = np.zeros((n, n), np.float32)
    g = [_gpu(a, device) for a in (uvw, freq, vis, wt, dirty0)]
    plan = GridderUvwEsFft(*g, px, px, eps, False)
    if cap is not None:
        plan.set_max_batch(cap)
    plan.grid_uvw_es_fft(*g)
    geo = es_oracle.geometry_for(uvw, freq, vis, dirty0, px, eps, False)
    ref = es_oracle.grid_uvw_es_fft(geo, uvw, freq, vis, wt, dirty0)
    return g[4].cpu().numpy(), ref


@pytest.mark.parametrize("rows,chan,n,eps,frac,order", [
    (20000, 8, 256, 1e-5, 0.45, "ascending"),
    (5000, 13, 256, 1e-5, 0.45, "descending"),
    (3000, 24, 256, 1e-5, 0.45, "shuffled"),     # non-monotonic channels
    (3000, 16, 128, 1e-5, 0.7, "ascending"),     # channels leave the grid
    (3000, 16, 256, 1e-7, 0.45, "ascending"),    # W = 16, 17-slot tables
    (40000, 64, 840, 0.05, 0.45, "ascending"),   # W = 4, G = 1024
])
def test_multichan_grid_matches_oracle(device, rows, chan, n, eps, frac, order):
    uvw, freq, vis, wt, px = make_case(21, rows, chan, n, frac=frac)
    freq = _order(freq, order, 22)
    out, ref = _grid(device, uvw, freq, vis, wt, n, px, eps)
    assert rel_l2(out, ref) < 1e-5


def test_multichan_integer_positions(device):
    """u = v = 0 rows: every channel at an exact integer position (W + 1
    taps), all channels of the row in one tile."""
    n = 128
    uvw, freq, vis, wt, px = make_case(23, 800, 10, n, frac=0.7)
    uvw[:40, :2] = 0.0
    out, ref = _grid(device, uvw, freq, vis, wt, n, px, 1e-5)
    assert rel_l2(out, ref) < 1e-5


def test_multichan_hot_tile_pieces(device):
    """All rows in the central tiles: > kPiece (4096) entries in a tile
    (several work items, combined by atomics into a zeroed tile)."""
    n = 256
    uvw, freq, vis, wt, px = make_case(24, 12000, 8, n, frac=0.01)
    out, ref = _grid(device, uvw, freq, vis, wt, n, px, 1e-5)
    assert rel_l2(out, ref) < 1e-5


def test_multichan_batched(device):
    """Row batches of a multi-channel call add their tiles to one grid."""
    n = 256
    uvw, freq, vis, wt, px = make_case(25, 9000, 16, n)
    out, ref = _grid(device, uvw, freq, vis, wt, n, px, 1e-5, cap=40000)
    assert rel_l2(out, ref) < 1e-5


def test_multichan_scatter_grid_cells(device):
    """The uv grid of the split API (sdp_grid_uvw_es_fft_scatter) cell by
    cell against the oracle's scatter."""
    import torch
    from ska_sdp_func.grid_data import GridderUvwEsFft

    n = 256
    uvw, freq, vis, wt, px = make_case(26, 3000, 12, n)
    freq = _order(freq, "shuffled", 27)
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
    assert len(bad) == 0, (len(bad), bad[:5])
