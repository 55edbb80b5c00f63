"""CPU oracle of the visibility weighting (TEST INFRASTRUCTURE ONLY: used by
tests/ as the checker, never by the product).

Restates src/ska-sdp-func/visibility/sdp_weighting.cpp (ska-sdp-func 1.2.2):
  cell of a visibility        :40-57  (idx = (int64)(floor(g / max * half)
                                        + half), skipped when >= grid_size)
  grid write                  :18-76  (grid[u][v][pol] += input weight)
  sums                        :80-137 (sum grid, sum (W)(grid * grid) over
                                        visibilities, in double)
  robustness                  :143-154
  uniform read                :158-217 (out = (W)(1.0 / grid))
  Briggs read                 :221-284 (out = (W)(in / (1 + R grid)))
Vectorised with numpy (grid write by np.add.at in visibility order, i.e.
the reference's summation order), plus a plain-loop version for tiny
inputs used to check the vectorised one. Negative cell indices (undefined
behaviour in the reference) are skipped, like the product.

Parity unpinned against reference outputs: the reference's tests for
this function hold no golden vectors and running reference code is
denied; checked against the plain-loop form and analytic
known answers (tests/).
"""
import numpy as np

C_0 = 299792458.0


def cells(uvw, freq_hz, max_abs_uv, grid_size):
    """(iu, iv, ok) for every (time, baseline, channel)."""
    inv_wl = freq_hz.astype(np.float64) / C_0                   # [C]
    gu = uvw[:, :, 0:1].astype(np.float64) * inv_wl             # [T, B, C]
    gv = uvw[:, :, 1:2].astype(np.float64) * inv_wl
    half = float(grid_size // 2)
    iu = (np.floor(gu / max_abs_uv * half) + half).astype(np.int64)
    iv = (np.floor(gv / max_abs_uv * half) + half).astype(np.int64)
    ok = (iu >= 0) & (iv >= 0) & (iu < grid_size) & (iv < grid_size)
    return iu, iv, ok


def weighting(uvw, freq_hz, max_abs_uv, grid, inp, out, robust=None):
    """In place on grid and out (numpy arrays); robust=None is uniform."""
    G = grid.shape[0]
    wt = grid.dtype.type
    iu, iv, ok = cells(uvw, freq_hz, max_abs_uv, G)
    T, B, C, P = inp.shape
    iu, iv, ok = iu.ravel(), iv.ravel(), ok.ravel()
    w_in = inp.reshape(-1, P)
    w_out = out.reshape(-1, P)
    for p in range(P):
        np.add.at(grid[:, :, p], (iu[ok], iv[ok]), w_in[ok, p])
    g = grid[iu[ok], iv[ok], :]                                  # [n, P]
    if robust is None:
        w_out[ok] = (1.0 / g.astype(np.float64)).astype(wt)
        return
    # Sequential sums in the reference's (visibility, polarisation) order
    # (cumsum accumulates left to right; np.sum would sum pairwise).
    s1 = float(np.cumsum(g.astype(np.float64).ravel())[-1]) if g.size else 0.0
    s2 = float(np.cumsum((g * g).astype(wt).astype(np.float64).ravel())[-1]) \
        if g.size else 0.0
    numer = (5.0 * 1 / (10.0 ** robust)) ** 2.0
    r = numer / (s2 / s1)
    w_out[ok] = (w_in[ok].astype(np.float64)
                 / (1.0 + r * g.astype(np.float64))).astype(wt)


def weighting_loops(uvw, freq_hz, max_abs_uv, grid, inp, out, robust=None):
    """Plain-loop restatement in the reference's loop order (tiny inputs)."""
    import math
    G = grid.shape[0]
    half = G // 2
    T, B, C, P = inp.shape
    wt = grid.dtype.type

    def cell(t, b, c):
        inv_wl = float(freq_hz[c]) / C_0
        u = float(uvw[t, b, 0]) * inv_wl
        v = float(uvw[t, b, 1]) * inv_wl
        i_u = int(math.floor(u / max_abs_uv * half) + half)
        i_v = int(math.floor(v / max_abs_uv * half) + half)
        if i_u < 0 or i_v < 0 or i_u >= G or i_v >= G:
            return None
        return i_u, i_v

    idx = [(t, b, c) for t in range(T) for b in range(B) for c in range(C)]
    for t, b, c in idx:
        k = cell(t, b, c)
        if k is None:
            continue
        for p in range(P):
            grid[k[0], k[1], p] += inp[t, b, c, p]
    r = 0.0
    if robust is not None:
        s1 = s2 = 0.0
        for t, b, c in idx:
            k = cell(t, b, c)
            if k is None:
                continue
            for p in range(P):
                g = grid[k[0], k[1], p]
                s1 += float(g)
                s2 += float(wt(g * g))
        r = (5.0 * 1 / (10.0 ** robust)) ** 2.0 / (s2 / s1)
    for t, b, c in idx:
        k = cell(t, b, c)
        if k is None:
            continue
        for p in range(P):
            g = float(grid[k[0], k[1], p])
            if robust is None:
                out[t, b, c, p] = wt(1.0 / g)
            else:
                out[t, b, c, p] = wt(float(inp[t, b, c, p]) / (1.0 + r * g))


# -- tiled Briggs weighting (sdp_opt_weighting) ------------------------------

def opt_briggs_runs(sorted_uu, sorted_vv, weights, sorted_tile, tile_offsets,
                    grid_size, robust, out, index=None):
    """sdp_optimized_weighting (index None: weights are the sorted weights,
    out is indexed by entry) / sdp_optimised_indexed_weighting (index =
    sorted_vis_index: weights and out indexed through it). Restates the
    per-run algorithm of sdp_opt_weighting.cu:21-126 / :131-273 with the
    reference's defects removed as include/ska-sdp-func/visibility/
    sdp_opt_weighting.h lists them: run b = [tile_offsets[b],
    tile_offsets[b + 1]) for b < num_tiles - 1, tile decoded from
    sorted_tile[start], cell = round(pos) + grid_size / 2 - tile origin,
    W = per-cell weight sums, R from sums over the run's in-tile entries.
    One plain loop per run (test sizes)."""
    tu, tv = 32, 16
    centre = grid_size // 2
    top_u = centre - (centre // tu) * tu - tu // 2
    top_v = centre - (centre // tv) * tv - tv // 2
    ntiles = ((grid_size + tu - 1) // tu) * ((grid_size + tv - 1) // tv)
    numerator = (5.0 * 1 / (10.0 ** robust)) ** 2
    wflat = weights.reshape(-1)
    oflat = out.reshape(-1)
    for b in range(ntiles - 1):
        s, e = int(tile_offsets[b]), int(tile_offsets[b + 1])
        if e <= s:
            continue
        code = int(sorted_tile[s])
        tile_u = (code & 32767) * tu + top_u
        tile_v = (code >> 15) * tv + top_v
        cells = []
        for i in range(s, e):
            gu = int(_cround(sorted_uu[i])) + centre - tile_u
            gv = int(_cround(sorted_vv[i])) + centre - tile_v
            if 0 <= gu < tu and 0 <= gv < tv:
                src = i if index is None else int(index[i])
                cells.append((i, gu * tv + gv, src))
        W = np.zeros(tu * tv)
        for _, c, src in cells:
            W[c] += wflat[src]
        sw = sum(W[c] for _, c, _ in cells)
        sw2 = sum(W[c] * W[c] for _, c, _ in cells)
        if not cells:
            continue
        rob = numerator / (sw2 / sw)
        for i, c, src in cells:
            oflat[src] = wflat[src] / (1 + rob * W[c])
    return out


def _cround(x):
    """C round(): half away from zero."""
    return np.sign(x) * np.floor(np.abs(x) + 0.5)


def briggs_global_test_reference(uvw, freqs, max_abs_uv, grid_size, robust,
                                 inp):
    """The reference test's own expected values for the indexed form
    (tests/visibility/test_opt_weighting.py:20-106 of the reference:
    reference_briggs_weights, a global Briggs weighting on a max_abs_uv
    grid), restated vectorised."""
    T, B, C, P = inp.shape
    out = np.zeros_like(inp)
    grid = np.zeros((grid_size, grid_size, P))
    f = freqs / C_0
    gu = uvw[:, :, 0:1] * f
    gv = uvw[:, :, 1:2] * f
    iu = (np.floor(gu / max_abs_uv * grid_size / 2) + grid_size / 2).astype(int)
    iv = (np.floor(gv / max_abs_uv * grid_size / 2) + grid_size / 2).astype(int)
    ok = (iu < grid_size) & (iv < grid_size)
    for p in range(P):
        np.add.at(grid[:, :, p], (iu[ok], iv[ok]), inp[..., p][ok])
    g = grid[iu.clip(max=grid_size - 1), iv.clip(max=grid_size - 1)]  # T,B,C,P
    sw = np.sum(np.where(ok[..., None], g, 0))
    sw2 = np.sum(np.where(ok[..., None], g * g, 0))
    rob = (5.0 * (1 / (10.0 ** robust))) ** 2 / (sw2 / sw)
    out = np.where(ok[..., None], inp / (1 + rob * g), out)
    return out
