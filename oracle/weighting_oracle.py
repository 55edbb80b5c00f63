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
