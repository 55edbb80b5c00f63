"""sdp_count_and_prefix_sum / sdp_bucket_sort / sdp_tiled_indexing
(csrc/visibility/sdp_tiled_functions.hip) against the CPU oracle
(oracle/tiled_oracle.py, the reference GPU kernels' arithmetic with entries
in visibility order). Integer outputs and the positions (computed with the
same operations) are compared exactly.
"""
import ctypes

import numpy as np
import pytest

from oracle import tiled_oracle as to

CELL = 1.0e-4


def make_case(T=3, B=60, C=4, P=1, dtype=np.float64, seed=5, spread=15000.0):
    rng = np.random.default_rng(seed)
    uvw = rng.uniform(-spread, spread, (T, B, 3)).astype(dtype)
    freqs = (1.0e8 + 2.0e6 * np.arange(C)).astype(dtype)
    vis = (rng.standard_normal((T, B, C, P)) +
           1j * rng.standard_normal((T, B, C, P))).astype(
        np.complex128 if dtype == np.float64 else np.complex64)
    weights = rng.uniform(0.5, 2.0, (T, B, C, P)).astype(dtype)
    return uvw, freqs, vis, weights


def test_oracle_geometry_and_known_tiles():
    g = to.geometry(1024, 32, 16, CELL)
    assert (g["ntu"], g["ntiles"], g["top_u"], g["top_v"]) == (32, 2048,
                                                               -16, -8)
    # uvw = 0 sits on the centre cell 512: rel_u = 528, support 4 ->
    # u tiles [floor(524/32), ceil(533/32)) = [16, 17); rel_v = 520 ->
    # v tiles [floor(516/16), ceil(525/16)) = [32, 33).
    uvw = np.zeros((1, 1, 3))
    _, _, pairs = to.tiles_of(uvw, np.array([1e8]), 0, 0, 0, 1024, 4, g)
    assert pairs == [(16, 32)]
    # A cell 2 below a u-tile boundary (gu = 527 -> rel 543): u tiles 16, 17.
    f = 1e8
    uvw[0, 0, 0] = 15.0 / (f / to.C_0 * 1024 * CELL)
    _, _, pairs = to.tiles_of(uvw, np.array([f]), 0, 0, 0, 1024, 4, g)
    assert pairs == [(16, 32), (17, 32)]


def test_oracle_sort_consistent_with_counts():
    uvw, freqs, vis, w = make_case()
    counts, offsets, skipped, total = to.count_and_prefix_sum(
        uvw, freqs, 4, 256, 32, 16, CELL, 4)
    assert skipped > 0 and total == counts.sum() > 0
    out, end = to.bucket_sort(uvw, freqs, vis, w, 256, 32, 16, CELL, 4,
                              offsets[:-1].tolist() + [offsets[-1]], total)
    np.testing.assert_array_equal(end[:-1], offsets[1:])
    # Each tile's slice holds entries of that tile (codes may carry a u
    # index one past either edge, which aliases into the neighbouring row).
    pv = (out["tile"].astype(np.int64) + 16384) // 32768
    pu = out["tile"] - pv * 32768
    flat = pu + pv * 8
    for k in range(len(counts)):
        assert np.all(flat[offsets[k]:offsets[k + 1]] == k)


def test_library_exports_tiled_functions():
    from ska_sdp_func.utility import Lib
    for n in ("sdp_count_and_prefix_sum", "sdp_bucket_sort",
              "sdp_tiled_indexing"):
        assert hasattr(Lib.handle(), n)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("tiles", [(32, 16), (10, 10)])
def test_gpu_matches_oracle(device, dtype, tiles):
    import torch
    from ska_sdp_func.visibility import (bucket_sort, count_and_prefix_sum,
                                         tiled_indexing)
    tu, tv = tiles
    grid, support, C = 256, 4, 4
    uvw, freqs, vis, w = make_case(C=C, dtype=dtype)
    counts, offsets, skipped, total = to.count_and_prefix_sum(
        uvw, freqs, C, grid, tu, tv, CELL, support)
    g = to.geometry(grid, tu, tv, CELL)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
    d_uvw, d_f, d_vis, d_w = d(uvw), d(freqs), d(vis), d(w)
    d_off = torch.full((g["ntiles"] + 1,), 7, dtype=torch.int32, device=device)
    d_cnt = torch.full((g["ntiles"],), 7, dtype=torch.int32, device=device)
    d_sk = torch.full((1,), 7, dtype=torch.int32, device=device)
    n = ctypes.c_int(0)
    count_and_prefix_sum(d_uvw, d_f, d_vis, grid, tu, tv, CELL, support, n,
                         d_off, d_cnt, d_sk)
    assert n.value == total
    np.testing.assert_array_equal(d_cnt.cpu().numpy(), counts)
    np.testing.assert_array_equal(d_off.cpu().numpy(), offsets)
    assert int(d_sk.cpu()[0]) == skipped
    # Bucket sort from those offsets.
    want, end = to.bucket_sort(uvw, freqs, vis, w, grid, tu, tv, CELL,
                               support, offsets, total)
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    outs = [torch.full((total,), 3, dtype=tdt, device=device)
            for _ in range(4)]
    s_tile = torch.full((total,), 3, dtype=torch.int32, device=device)
    bucket_sort(d_uvw, d_f, d_vis, d_w, grid, tu, tv, CELL, support,
                outs[0], outs[1], outs[2], s_tile, outs[3], d_off)
    got = dict(uu=outs[0], vv=outs[1], weight=outs[2], tile=s_tile,
               vis=outs[3])
    for k, v in got.items():
        np.testing.assert_array_equal(v.cpu().numpy(), want[k], err_msg=k)
    np.testing.assert_array_equal(d_off.cpu().numpy(), end)
    # Tiled indexing from fresh offsets.
    d_off2 = d(offsets.astype(np.int32))
    want, end = to.bucket_sort(uvw, freqs, None, None, grid, tu, tv, CELL,
                               support, offsets, total, indexed=True,
                               num_channels=C)
    uu = torch.zeros((total,), dtype=tdt, device=device)
    vv = torch.zeros((total,), dtype=tdt, device=device)
    tl = torch.zeros((total,), dtype=torch.int32, device=device)
    vi = torch.zeros((total,), dtype=torch.int32, device=device)
    T, B = uvw.shape[:2]
    tiled_indexing(d_uvw, d_f, grid, tu, tv, CELL, support, C, B, T, tl, uu,
                   vv, vi, d_off2)
    for k, v in dict(uu=uu, vv=vv, tile=tl, vis_index=vi).items():
        np.testing.assert_array_equal(v.cpu().numpy(), want[k], err_msg=k)
    np.testing.assert_array_equal(d_off2.cpu().numpy(), end)


@pytest.mark.gpu
def test_gpu_errors(device):
    from ska_sdp_func.utility import CError
    from ska_sdp_func.visibility import count_and_prefix_sum
    uvw, freqs, vis, w = make_case()
    off = np.zeros(8 * 16 + 1, np.int32)
    with pytest.raises(CError, match="Memory location mismatch"):
        count_and_prefix_sum(uvw, freqs, vis, 256, 32, 16, CELL, 4,
                             ctypes.c_int(0), off, off[:-1].copy(),
                             np.zeros(1, np.int32))


@pytest.mark.gpu
def test_gpu_undersized_sorted_arrays_rejected(device):
    """Sorted arrays shorter than the entries (or caller offsets running past
    them) give SDP_ERR_INVALID_ARGUMENT and leave the cursors untouched,
    instead of a truncated sort with advanced cursors."""
    import torch
    from ska_sdp_func.utility import CError
    from ska_sdp_func.visibility import tiled_indexing
    grid, support, C, tu, tv = 256, 4, 4, 32, 16
    uvw, freqs, vis, w = make_case(C=C)
    counts, offsets, skipped, total = to.count_and_prefix_sum(
        uvw, freqs, C, grid, tu, tv, CELL, support)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
    T, B = uvw.shape[:2]
    for cap, off in ((total - 1, offsets),
                     (total, offsets + np.int32(1))):
        d_off = d(off.astype(np.int32))
        arrs = [torch.zeros((cap,), dtype=torch.float64, device=device)
                for _ in range(2)]
        ints = [torch.zeros((cap,), dtype=torch.int32, device=device)
                for _ in range(2)]
        with pytest.raises(CError, match="Invalid function argument"):
            tiled_indexing(d(uvw), d(freqs), grid, tu, tv, CELL, support, C,
                           B, T, ints[0], arrs[0], arrs[1], ints[1], d_off)
        np.testing.assert_array_equal(d_off.cpu().numpy(), off)
