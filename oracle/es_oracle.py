"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the ES-FFT (de)gridder.

A restatement of the reference pipeline of ska-sdp-func 1.2.2
  sdp_grid_uvw_es_fft       src/ska-sdp-func/grid_data/sdp_gridder_uvw_es_fft.cpp:532-742
  sdp_ifft_degrid_uvw_es    src/ska-sdp-func/grid_data/sdp_gridder_uvw_es_fft.cpp:745-956
with the per-visibility scatter/gather in C (oracle/es_oracle.c), and the
FFT, w-screen and convolution correction in numpy (float64):
  apply_w_screen_and_sum    sdp_gridder_uvw_es_fft_kernels.cu:429-547
  reverse_w_screen_to_stack sdp_gridder_uvw_es_fft_kernels.cu:554-679
  conv_corr_and_scaling     sdp_gridder_uvw_es_fft_kernels.cu:690-769
  phase_shift / conv_corr   sdp_gridder_uvw_es_fft_kernels.cu:69-87, 110-123
FFT: unnormalised C2C, inverse (+i) for gridding, forward (-i) for
degridding, as cuFFT is driven at sdp_fft.cpp:883-921.

Used ONLY by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
as the checker. The product library never imports this.

Parity status: the reference ES path is GPU-only (CUDA) and cannot run here,
so absolute dirty-image / visibility values of this path are pinned by:
  * the parameter tables (tests/golden/es_params.json) produced by the
    reference's own host code compiled in oracle/_ref;
  * a direct DFT of the same visibilities (tests/test_oracle.py), which the
    ES gridder must approximate to its epsilon;
  * the reference test suite's adjointness recipe
    (tests/grid_data/test_gridder_uvw_es_fft.py:532-637 of the reference).
"""
import ctypes
import math
import os
import subprocess

import numpy as np

from . import es_params

from . import _cc

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def build(force=False):
    """Compile oracle/es_oracle.c (gcc, OpenMP) (oracle/_cc.py)."""
    return _cc.shared("es_oracle.c", "libes_oracle.so",
                      ["-O2", "-fopenmp", "-fno-fast-math", "-ffp-contract=off"],
                      force)


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
        P = ctypes.c_void_p
        i64, i32 = ctypes.c_int64, ctypes.c_int
        f32, f64 = ctypes.c_float, ctypes.c_double
        _lib.oracle_es_grid_f32.argtypes = [i64, i32, P, P, P, P, i32, i32,
                                            f32, f32, f32, f32, i32, i32, P]
        _lib.oracle_es_grid_f64.argtypes = [i64, i32, P, P, P, P, i32, i32,
                                            f64, f64, f64, f64, i32, i32, P]
        _lib.oracle_es_degrid_f32.argtypes = [i64, i32, P, P, P, i32, i32,
                                              f32, f32, f32, f32, i32, i32,
                                              P]
        _lib.oracle_es_degrid_f64.argtypes = [i64, i32, P, P, P, i32, i32,
                                              f64, f64, f64, f64, i32, i32,
                                              P]
        _lib.oracle_es_grid_f32_omp.argtypes = [i64, i32, P, P, P, P, i32,
                                                i32, f32, f32, P]
        _lib.oracle_es_grid_f32_omp.restype = i32
        _lib.oracle_set_threads.argtypes = [i32]
        _lib.oracle_set_threads.restype = i32
        _lib.oracle_es_grid_f32_par.argtypes = \
            _lib.oracle_es_grid_f32.argtypes
        _lib.oracle_es_grid_f32_par.restype = i32
        _lib.oracle_es_grid_f64_par.argtypes = \
            _lib.oracle_es_grid_f64.argtypes
        _lib.oracle_es_grid_f64_par.restype = i32
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _is_double(vis):
    return vis.dtype == np.complex128


def geometry_for(uvw, freq, vis, dirty, pixel_size, epsilon, do_w):
    """Plan geometry as GridderUvwEsFft.__init__ + create_plan derive it."""
    min_w = max_w = 0.0
    if do_w:
        # gridder_uvw_es_fft.py:90-106
        min_w = float(np.amin(np.abs(uvw[:, 2]))) * float(freq[0]) / 299792458.0
        max_w = float(np.amax(np.abs(uvw[:, 2]))) * float(freq[-1]) / 299792458.0
    return es_params.plan_geometry(dirty.shape[0], pixel_size, epsilon,
                                   _is_double(vis), do_w, min_w, max_w)


def _precision_args(geo, dbl):
    cast = float if dbl else (lambda x: float(np.float32(x)))
    return (cast(geo["beta"]), cast(geo["uv_scale"]), cast(geo["w_scale"]),
            cast(geo["min_plane_w"]))


def _pixel_offsets(n):
    """Signed pixel offsets x in [-half, half-1] and image indices."""
    half = n // 2
    off = np.arange(-half, half)
    return off, off + half


def correction_map(geo, rt=np.float64):
    """1/correction per pixel offset [y][x], conv_corr_and_scaling
    (kernels.cu:690-769), in the working precision rt of the reference path
    (the cos() argument is double there, as its double PI literal promotes
    it)."""
    n = geo["image_size"]
    off, _ = _pixel_offsets(n)
    a = np.abs(off)
    cc = geo["conv_corr"].astype(rt)
    norm = rt(geo["conv_corr_norm"])
    lconv = cc[a][None, :]       # column offset x -> l
    mconv = cc[a][:, None]       # row offset y -> m
    if geo["do_w"]:
        px = rt(geo["pixel_size"])
        l = px * a[None, :].astype(rt)
        m = px * a[:, None].astype(rt)
        nn = np.sqrt(rt(1) - l * l - m * m) - rt(1)
        k = nn * rt(geo["inv_w_scale"])
        supp = geo["support"]
        p = int(math.ceil(1.5 * supp + 2.0))
        qk = geo["quad_kernel"].astype(rt).astype(np.float64)
        qn = geo["quad_nodes"].astype(rt).astype(np.float64)
        qw = geo["quad_weights"].astype(rt).astype(np.float64)
        acc = np.zeros(nn.shape, dtype=rt)
        for i in range(p):
            term = qk[i] * np.cos(np.pi * k.astype(np.float64) * supp * qn[i]) * qw[i]
            acc = (acc.astype(np.float64) + term).astype(rt)
        nconv = acc * rt(supp)
        nconv = nconv * (norm * norm)
        corr = lconv * mconv * nconv
    else:
        corr = lconv * mconv * norm * norm
    return rt(1) / corr


def _phasor(geo, plane, sign, rt=np.float64):
    """phase_shift(w, l, m, sign) on the [y][x] offset grid (:110-123)."""
    n = geo["image_size"]
    off, _ = _pixel_offsets(n)
    a = np.abs(off)
    px = rt(geo["pixel_size"])
    l = px * a[None, :].astype(rt)
    m = px * a[:, None].astype(rt)
    sos = l * l + m * m
    nm1 = (-sos) / (np.sqrt(rt(1) - sos) + rt(1))
    w = rt(plane) * rt(geo["inv_w_scale"]) + rt(geo["min_plane_w"])
    x = rt(2) * rt(np.pi) * w * nm1
    xn = rt(1) / (nm1 + rt(1))
    return np.cos(rt(sign) * x) * xn, np.sin(rt(sign) * x) * xn


def _checker(n):
    off, _ = _pixel_offsets(n)
    return np.where(((off[:, None] + off[None, :]) & 1) != 0, -1.0, 1.0)


def scatter(geo, uvw, freq, vis, weight, plane=0):
    """Grid (before FFT) of one w-plane, complex128 [G][G]."""
    G = geo["grid_size"]
    grid = np.zeros((G, G), dtype=np.complex128)
    dbl = _is_double(vis)
    beta, uvs, ws, mpw = _precision_args(geo, dbl)
    R, C = vis.shape
    uvw = np.ascontiguousarray(uvw)
    freq = np.ascontiguousarray(freq)
    vis = np.ascontiguousarray(vis)
    weight = np.ascontiguousarray(weight)
    # Stripe-parallel form: the same taps and, per cell, the same summation
    # order as the serial oracle_es_grid_f32/_f64 (es_oracle.c).
    fn = (lib().oracle_es_grid_f64_par if dbl
          else lib().oracle_es_grid_f32_par)
    fn(R, C, _ptr(uvw), _ptr(freq), _ptr(vis), _ptr(weight), G,
       geo["support"], beta, uvs, ws, mpw, int(geo["do_w"]), plane,
       _ptr(grid))
    return grid


def gather(geo, uvw, freq, grid, out_vis, plane=0):
    """out_vis (complex128 [R][C]) += taps(one w-plane) * grid."""
    G = geo["grid_size"]
    dbl = uvw.dtype == np.float64
    beta, uvs, ws, mpw = _precision_args(geo, dbl)
    R, C = out_vis.shape
    grid = np.ascontiguousarray(grid, dtype=np.complex128)
    fn = lib().oracle_es_degrid_f64 if dbl else lib().oracle_es_degrid_f32
    fn(R, C, _ptr(np.ascontiguousarray(uvw)),
       _ptr(np.ascontiguousarray(freq)), _ptr(grid), G, geo["support"],
       beta, uvs, ws, mpw, int(geo["do_w"]), plane, _ptr(out_vis))


def _workers():
    return int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1


def _ifft2(grid):
    """Unnormalised inverse 2-D FFT in float64 (pocketfft, threaded)."""
    try:
        import scipy.fft
        return scipy.fft.ifft2(grid, norm="forward", workers=_workers())
    except ImportError:
        return np.fft.ifft2(grid, norm="forward")


def _fft2(grid):
    """Unnormalised forward 2-D FFT in float64 (pocketfft, threaded)."""
    try:
        import scipy.fft
        return scipy.fft.fft2(grid, workers=_workers())
    except ImportError:
        return np.fft.fft2(grid)


def _rt(dirty_or_vis):
    dt = np.asarray(dirty_or_vis).dtype
    return np.float64 if dt in (np.float64, np.complex128) else np.float32


def grid_uvw_es_fft(geo, uvw, freq, vis, weight, dirty_in):
    """dirty_out = (dirty_in + sum_planes screen(IFFT(scatter))) * corr.

    Image-plane arithmetic (screen, phasor, accumulation, correction) is
    done in the reference's working precision; the FFT in float64.
    """
    rt = _rt(vis)
    n = geo["image_size"]
    G = geo["grid_size"]
    half, gc = n // 2, G // 2
    sl = slice(gc - half, gc + half)
    dirty = np.array(dirty_in, dtype=rt, copy=True)
    sgn = _checker(n).astype(rt)
    for plane in range(geo["num_w_planes"]):
        grid = scatter(geo, uvw, freq, vis, weight, plane)
        layer = _ifft2(grid)                            # unnormalised, +i
        sub = layer[sl, sl]
        re = sub.real.astype(rt)
        im = sub.imag.astype(rt)
        if geo["do_w"]:
            pr, pi = _phasor(geo, plane, -1.0, rt)
            val = re * pr - im * pi
        else:
            val = re
        dirty[:2 * half, :2 * half] += sgn * val
    dirty[:2 * half, :2 * half] *= correction_map(geo, rt)
    return dirty


def ifft_degrid_uvw_es(geo, uvw, freq, dirty_in, num_chan=None):
    """(vis_out complex128 [R][C], dirty after in-place correction)."""
    rt = _rt(dirty_in)
    n = geo["image_size"]
    G = geo["grid_size"]
    half, gc = n // 2, G // 2
    dirty = np.array(dirty_in, dtype=rt, copy=True)
    dirty[:2 * half, :2 * half] *= correction_map(geo, rt)
    sgn = _checker(n).astype(rt)
    R = uvw.shape[0]
    C = num_chan if num_chan is not None else len(freq)
    out = np.zeros((R, C), dtype=np.complex128)
    sl = slice(gc - half, gc + half)
    img = sgn * dirty[:2 * half, :2 * half]
    for plane in range(geo["num_w_planes"]):
        grid = np.zeros((G, G), dtype=np.complex128)
        if geo["do_w"]:
            pr, pi = _phasor(geo, plane, 1.0, rt)
            grid[sl, sl] = (pr * img).astype(np.float64) + 1j * (
                pi * img).astype(np.float64)
        else:
            grid[sl, sl] = img
        grid = _fft2(grid)                               # unnormalised, -i
        gather(geo, uvw, freq, grid, out, plane)
    return out, dirty


def dft_dirty(uvw, freq, vis, weight, n, pixel_size, do_w=False):
    """Direct (slow) dirty image, the quantity the ES gridder approximates:
        I[y][x] = Re sum_k w_k V_k exp(2 pi i (u_k m_y + v_k l_x
                                        - w_k (n_yx - 1))) / n_yx
    (2-D: the w term and 1/n are dropped). Row index <-> u, column <-> v.
    Used to pin the oracle's absolute values independently of the reference.
    """
    half = n // 2
    off = np.arange(-half, half) * pixel_size
    out = np.zeros((n, n))
    R, C = vis.shape
    if do_w:
        nn = np.sqrt(1.0 - off[None, :] ** 2 - off[:, None] ** 2)
    for c in range(C):
        s = float(freq[c]) / 299792458.0
        u = uvw[:, 0].astype(np.float64) * s
        v = uvw[:, 1].astype(np.float64) * s
        wv = (vis[:, c] * weight[:, c]).astype(np.complex128)
        if not do_w:
            eu = np.exp(2j * np.pi * np.outer(off, u))      # [n][R]
            ev = np.exp(2j * np.pi * np.outer(off, v))      # [n][R]
            out += ((eu * wv[None, :]) @ ev.T).real
        else:
            w = uvw[:, 2].astype(np.float64) * s
            for k in range(R):
                ph = np.exp(2j * np.pi * (off[:, None] * u[k] + off[None, :]
                                          * v[k] - w[k] * (nn - 1.0)))
                out += (wv[k] * ph / nn).real
    return out


def dft_degrid(uvw, freq, dirty, pixel_size, do_w=False):
    """Adjoint of dft_dirty: V_k = sum_yx I[y][x] exp(-2 pi i (...)) / n."""
    n = dirty.shape[0]
    half = n // 2
    off = np.arange(-half, half) * pixel_size
    img = np.asarray(dirty[:2 * half, :2 * half], dtype=np.float64)
    if do_w:
        nn = np.sqrt(1.0 - off[None, :] ** 2 - off[:, None] ** 2)
    R, C = uvw.shape[0], len(freq)
    out = np.zeros((R, C), dtype=np.complex128)
    for c in range(C):
        s = float(freq[c]) / 299792458.0
        for k in range(R):
            u, v, w = (float(x) * s for x in uvw[k])
            ph = np.exp(-2j * np.pi * (off[:, None] * u + off[None, :] * v))
            if do_w:
                ph = ph * np.exp(2j * np.pi * w * (nn - 1.0)) / nn
            out[k, c] = np.sum(img * ph)
    return out
