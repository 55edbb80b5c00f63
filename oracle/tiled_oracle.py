"""CPU restatement of the reference visibility tiling / bucket sort
(TEST INFRASTRUCTURE: only tests/ may use this module, as the checker; the
product path never imports it).

Follows the reference GPU kernels, src/ska-sdp-func/visibility/
sdp_tiled_functions.cu of ska-sdp-func 1.2.2:
  geometry        sdp_tiled_functions.cpp:331-342 (tile counts, top-left)
  position/tiles  .cu:91-114 (pos = uvw * (f / c0) * grid_size * cell in
                  the uvw precision, C round, support test, float tile
                  bounds floor((rel - support) / tile), ceil((rel + support
                  + 1) / tile))
  bucket sort     .cu:191-207 (entry -> tile_offsets[tile]++, sorted_tile
                  = pv * 32768 + pu, vis / weight element (t, b, c) of the
                  arrays read as reals of the uvw precision)
Entries inside a tile in visibility order (the deterministic order the HIP
path produces; the reference's atomics leave it arbitrary), tile indices
outside [0, num_tiles) dropped (the reference writes them out of bounds).

Parity unpinned against reference outputs: the reference test
(tests/visibility/test_tiled_functions.py) only checks the total count and
compares `.all()` booleans, and its CPU path computes a different function
(tile_v_min passed in the u-minimum slot, sdp_tiled_functions.cpp:84-89).
Checked against hand-derived tile sets in tests/test_tiled_functions.py.
"""
import math

import numpy as np

C_0 = 299792458.0


def geometry(grid, tu, tv, cell):
    centre = grid // 2
    ntu = (grid + tu - 1) // tu
    ntv = (grid + tv - 1) // tv
    top_u = centre - (centre // tu) * tu - tu // 2
    top_v = centre - (centre // tv) * tv - tv // 2
    return dict(ntu=ntu, ntiles=ntu * ntv, top_u=top_u, top_v=top_v,
                inv_tu=np.float32(1.0 / tu), inv_tv=np.float32(1.0 / tv),
                grid_scale=grid * cell, centre=centre)


def _cround(x):
    x = float(x)
    return int(math.copysign(math.floor(abs(x) + 0.5), x))


def tiles_of(uvw, freqs, t, b, c, grid, support, g):
    """(pos_u, pos_v, [(pu, pv), ...]) or (pos_u, pos_v, None) if skipped."""
    U = uvw.dtype.type
    inv_wl = U(float(freqs[c]) / C_0)
    pos_u = U(float(U(uvw[t, b, 0] * inv_wl)) * g["grid_scale"])
    pos_v = U(float(U(uvw[t, b, 1] * inv_wl)) * g["grid_scale"])
    gu = _cround(pos_u) + g["centre"]
    gv = _cround(pos_v) + g["centre"]
    if not (gu + support < grid and gu - support >= 0 and
            gv + support < grid and gv - support >= 0):
        return pos_u, pos_v, None
    f32 = np.float32
    rel_u, rel_v = gu - g["top_u"], gv - g["top_v"]
    u1 = f32(f32(rel_u - support) * g["inv_tu"])
    u2 = f32(f32(rel_u + support + 1) * g["inv_tu"])
    v1 = f32(f32(rel_v - support) * g["inv_tv"])
    v2 = f32(f32(rel_v + support + 1) * g["inv_tv"])
    pairs = [(pu, pv) for pv in range(math.floor(v1), math.ceil(v2))
             for pu in range(math.floor(u1), math.ceil(u2))]
    return pos_u, pos_v, pairs


def _entries(uvw, freqs, C, grid, support, g):
    T, B = uvw.shape[:2]
    for t in range(T):
        for b in range(B):
            for c in range(C):
                v = (t * B + b) * C + c
                pu, pv, pairs = tiles_of(uvw, freqs, t, b, c, grid, support,
                                         g)
                yield v, pu, pv, pairs


def count_and_prefix_sum(uvw, freqs, C, grid, tu, tv, cell, support):
    """(num_points_in_tiles, tile_offsets, num_skipped, total)."""
    g = geometry(grid, tu, tv, cell)
    counts = np.zeros(g["ntiles"], np.int32)
    skipped = 0
    for _, _, _, pairs in _entries(uvw, freqs, C, grid, support, g):
        if pairs is None:
            skipped += 1
            continue
        for a, b in pairs:
            k = a + b * g["ntu"]
            if 0 <= k < g["ntiles"]:
                counts[k] += 1
    offsets = np.zeros(g["ntiles"] + 1, np.int32)
    offsets[1:] = np.cumsum(counts)
    return counts, offsets, skipped, int(offsets[-1])


def bucket_sort(uvw, freqs, vis, weights, grid, tu, tv, cell, support,
                tile_offsets, n_out, indexed=False, num_channels=None):
    """Sorted arrays (dict) and the advanced tile_offsets."""
    g = geometry(grid, tu, tv, cell)
    U = uvw.dtype.type
    C = vis.shape[2] if num_channels is None else num_channels
    per_tile = [[] for _ in range(g["ntiles"])]
    for v, pu, pv, pairs in _entries(uvw, freqs, C, grid, support, g):
        if pairs is None:
            continue
        for a, b in pairs:
            k = a + b * g["ntu"]
            if 0 <= k < g["ntiles"]:
                per_tile[k].append((v, pu, pv, b * 32768 + a))
    out = dict(uu=np.zeros(n_out, U), vv=np.zeros(n_out, U),
               tile=np.zeros(n_out, np.int32))
    if indexed:
        out["vis_index"] = np.zeros(n_out, np.int32)
    else:
        out["vis"] = np.zeros(n_out, U)
        out["weight"] = np.zeros(n_out, U)
        vis_flat = np.ascontiguousarray(vis).view(U).ravel()
        w_flat = np.ascontiguousarray(weights).ravel()
    offsets = np.array(tile_offsets, np.int64)
    for k, lst in enumerate(per_tile):
        for rank, (v, pu, pv, code) in enumerate(lst):
            pos = offsets[k] + rank
            if not 0 <= pos < n_out:
                continue
            out["uu"][pos], out["vv"][pos], out["tile"][pos] = pu, pv, code
            if indexed:
                out["vis_index"][pos] = v
            else:
                out["vis"][pos] = vis_flat[v]
                out["weight"][pos] = w_flat[v]
        offsets[k] += len(lst)
    return out, offsets.astype(np.int32)
