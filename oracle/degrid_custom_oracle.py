"""CPU oracle of sdp_degrid_uvw_custom (TEST INFRASTRUCTURE ONLY: used by
tests/ as the checker, never by the product).

Restates src/ska-sdp-func/grid_data/sdp_degrid_uvw_custom.cpp (ska-sdp-func
1.2.2): calculate_coordinates :20-62 (C round: half away from zero),
in-grid test :134-140, the nested x / y / z sums :143-176 in that order,
conjugation :177, output only for in-grid visibilities. A vectorised form
(numpy over visibilities) and a plain-loop form for tiny inputs.

Parity unpinned against reference outputs: the reference's tests for
this function hold no golden vectors and running reference code is
denied; checked against the plain-loop form and analytic
known answers (tests/).
"""
import numpy as np

C_0 = 299792458.0


def _round_c(x):
    return np.sign(x) * np.floor(np.abs(x) + 0.5)


def coordinates(u, v, w, X, os_, osw, theta, wstep):
    iox = (_round_c(theta * u * os_)).astype(np.int64) + (X // 2 + 1) * os_ - 1
    ioy = (_round_c(theta * v * os_)).astype(np.int64) + (X // 2 + 1) * os_ - 1
    ioz = (_round_c((1.0 + w / wstep) * osw)).astype(np.int64) + osw - 1
    # C integer division / remainder truncate toward zero.
    home_x = np.trunc(iox / os_).astype(np.int64)
    home_y = np.trunc(ioy / os_).astype(np.int64)
    frac_x = os_ - 1 - np.fmod(iox, os_)
    frac_y = os_ - 1 - np.fmod(ioy, os_)
    frac_z = osw - 1 - np.fmod(ioz, osw)
    return home_x, home_y, frac_x, frac_y, frac_z


def degrid(grid, uvw, uv_kernel, w_kernel, theta, wstep, f0, df, conjugate,
           vis):
    """In place on vis (numpy complex128 [T, B, C, P])."""
    C, Z, Y, X, P = grid.shape
    os_, K = uv_kernel.shape
    osw, KW = w_kernel.shape
    T, B = uvw.shape[:2]
    half = K // 2
    inv_wl = (f0 + np.arange(C) * df) / C_0
    u = uvw[:, :, 0:1] * inv_wl
    v = uvw[:, :, 1:2] * inv_wl
    w = uvw[:, :, 2:3] * inv_wl
    hx, hy, fx, fy, fz = coordinates(u, v, w, X, os_, osw, theta, wstep)
    ok = (hx > half) & (hx < X - half) & (hy > half) & (hy < Y - half)
    # w-kernel rows past the table (negative ioz, reference reads out of
    # bounds): left unwritten, as the HIP kernel does.
    ok &= fz < osw
    t_i, b_i, c_i = np.nonzero(ok)
    hx, hy = hx[ok], hy[ok]
    ku = uv_kernel[fx[ok]]            # [n, K]
    kv = uv_kernel[fy[ok]]
    kw = w_kernel[fz[ok]]             # [n, KW]
    ys = hy[:, None] + np.arange(K)[None, :] - half
    xs = hx[:, None] + np.arange(K)[None, :] - half
    g = grid[c_i[:, None, None, None], np.arange(KW)[None, :, None, None],
             ys[:, None, :, None], xs[:, None, None, :], :]   # [n, Z, Y, X, P]
    visy = np.einsum("nzyxp,nx->nzyp", g, ku)
    visz = np.einsum("nzyp,ny->nzp", visy, kv)
    out = np.einsum("nzp,nz->np", visz, kw)
    if conjugate:
        out = np.conj(out)
    vis[t_i, b_i, c_i, :] = out


def degrid_loops(grid, uvw, uv_kernel, w_kernel, theta, wstep, f0, df,
                 conjugate, vis):
    import math
    C, Z, Y, X, P = grid.shape
    os_, K = uv_kernel.shape
    osw, KW = w_kernel.shape
    T, B = uvw.shape[:2]
    half = K // 2

    def rnd(x):
        return int(math.copysign(math.floor(abs(x) + 0.5), x))

    def cdiv(a, b):
        return int(a / b) if a >= 0 else -((-a) // b)

    def cmod(a, b):
        return a - cdiv(a, b) * b

    for t in range(T):
        for b in range(B):
            for c in range(C):
                iw = (f0 + c * df) / C_0
                u, v, w = (iw * uvw[t, b, 0], iw * uvw[t, b, 1],
                           iw * uvw[t, b, 2])
                iox = rnd(theta * u * os_) + (X // 2 + 1) * os_ - 1
                ioy = rnd(theta * v * os_) + (X // 2 + 1) * os_ - 1
                ioz = rnd((1.0 + w / wstep) * osw) + osw - 1
                hx, hy = cdiv(iox, os_), cdiv(ioy, os_)
                fx = os_ - 1 - cmod(iox, os_)
                fy = os_ - 1 - cmod(ioy, os_)
                fz = osw - 1 - cmod(ioz, osw)
                if not (half < hx < X - half and half < hy < Y - half):
                    continue
                if fz >= osw:
                    continue
                for p in range(P):
                    acc = 0j
                    for z in range(KW):
                        vz = 0j
                        for y in range(K):
                            vy = 0j
                            for x in range(K):
                                vy += uv_kernel[fx, x] * grid[
                                    c, z, hy + y - half, hx + x - half, p]
                            vz += uv_kernel[fy, y] * vy
                        acc += w_kernel[fz, z] * vz
                    vis[t, b, c, p] = acc.conjugate() if conjugate else acc
