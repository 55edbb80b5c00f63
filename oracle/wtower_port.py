"""TEST INFRASTRUCTURE ONLY -- driver of oracle/wtower_port.c, the C/OpenMP
port of the reference CPU path of sdp_grid_wstack_wtower_grid_all
(sdp_grid_wstack_wtower.cpp:475-736). Used by bench_wtower.py's
cpu_baseline leg (timed on the GPU box's host cores) and checked against
the numpy restatement (oracle/wtower_oracle.py) in
tests/test_wtower_port.py. Never imported by the product package.

Per w-stack plane the C code does what the reference's plane loop does:
clamp rows to the plane, bin them to sub-grid tasks, grid every task
through the w-tower (layer by layer, one sub-grid FFT per layer) on the
OpenMP threads, FFT each sub-grid and add it to the plane grid under a
critical section (port_grid_plane); then the plane FFT, the PSWF / w-stack
grid correction and the accumulation into the image (port_finish_plane).
The set-up the reference does once per call (kernel tables, w-pattern,
PSWF tables, bounds) is done here in numpy.
"""
import ctypes
import math
import os
import subprocess

import numpy as np

from . import wtower_oracle as wo

from . import _cc

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None
C_0 = 299792458.0


def build(force=False):
    """Compile oracle/wtower_port.c (gcc -O3, OpenMP) (oracle/_cc.py)."""
    return _cc.shared("wtower_port.c", "libwtower_port.so",
                      ["-O3", "-fcx-limited-range", "-fopenmp"],
                      force)


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
        P, i32, i64, f64 = (ctypes.c_void_p, ctypes.c_int, ctypes.c_int64,
                            ctypes.c_double)
        _lib.port_set_threads.argtypes = [i32]
        _lib.port_set_threads.restype = i32
        _lib.port_grid_plane.argtypes = [
            i64, i32, P, P, f64, f64, i32, i32, f64, f64, i32, i32, i32, i32,
            P, P, P, f64, f64, i64, i64, i64, i64, i64, P, i64, i64, P]
        _lib.port_grid_plane.restype = i64
        _lib.port_finish_plane.argtypes = [
            i32, P, P, f64, f64, f64, f64, i32, P, P, i32, f64]
        _lib.port_finish_plane.restype = i32
    return _lib


def set_threads(n):
    return int(lib().port_set_threads(int(n)))


def pswf_legendre(c, num_terms=40):
    """Legendre coefficients d_0, d_2, ... of S_00(c, x) (Flammer
    normalisation, S(0) = 1): the lowest eigenvector of the three-term
    recurrence of the prolate equation in the Legendre basis (m = 0), the
    expansion sdp_pswf_aswfa sums (sdp_pswf.cpp)."""
    r = 2 * np.arange(num_terms, dtype=np.float64)
    c2 = c * c
    a = (r + 2) * (r + 1) * c2 / ((2 * r + 3) * (2 * r + 5))
    b = r * (r + 1) + c2 * (2 * r * (r + 1) - 1) / ((2 * r - 1) * (2 * r + 3))
    with np.errstate(divide="ignore", invalid="ignore"):
        g = np.where(r > 0, r * (r - 1) * c2 / ((2 * r - 3) * (2 * r - 1)),
                     0.0)
    m = np.diag(b) + np.diag(a[:-1], 1) + np.diag(g[1:], -1)
    lam, vec = np.linalg.eig(m)
    d = np.real(vec[:, np.argmin(np.real(lam))])
    # P_{2k}(0) = (-1)^k (2k-1)!! / (2k)!!
    p0 = np.ones(num_terms)
    for k in range(1, num_terms):
        p0[k] = -p0[k - 1] * (2 * k - 1) / (2 * k)
    d = d / np.dot(d, p0)
    # drop the tail below double precision
    keep = np.nonzero(np.abs(d) > 1e-18 * np.abs(d[0]))[0]
    return d[:keep[-1] + 1]


def _bounds(uvw, f0, df, C):
    """uvw_bounds_all over every (row, channel), vectorised."""
    a = uvw * (f0 / C_0)
    b = uvw * ((f0 + (C - 1) * df) / C_0)
    return np.minimum(a, b).min(0), np.maximum(a, b).max(0)


class Plan:
    """Everything grid_all sets up once per call (grid_all :532-612)."""

    def __init__(self, vis, f0, df, uvw, N, S, theta, w_step, support,
                 oversampling, w_support, w_oversampling, subgrid_frac, H):
        self.vis = np.ascontiguousarray(vis, np.complex64)
        self.uvw = np.ascontiguousarray(uvw, np.float64)
        self.R, self.C = self.vis.shape
        self.f0, self.df = f0, (df if df != 0.0 else 10.0)
        self.N, self.S, self.theta, self.w_step = N, S, theta, w_step
        self.kw = (support, oversampling, w_support, w_oversampling)
        self.frac = subgrid_frac if subgrid_frac != 0.0 else 2.0 / 3.0
        self.H = H
        self.uv_kernel = np.ascontiguousarray(
            wo.make_pswf_kernel(support, oversampling))
        self.w_kernel = np.ascontiguousarray(
            wo.make_pswf_kernel(w_support, w_oversampling))
        self.w_pattern = np.ascontiguousarray(
            wo.make_w_pattern(S, theta, 0.0, 0.0, w_step))
        self.pswf_lm = np.ascontiguousarray(
            wo.generate_pswf(support * (np.pi / 2), N, True))
        self.c_n = w_support * (np.pi / 2)
        self.leg = np.ascontiguousarray(pswf_legendre(self.c_n))
        eff = int(math.floor(S * self.frac))
        eff_dist = eff / theta
        ws_dist = H * w_step
        lo, hi = _bounds(self.uvw, f0, self.df, self.C)
        eta = 1e-5
        rng = lambda x, y, d: (int(math.floor(x / d + 0.5 - eta)),
                               int(math.floor(y / d + 0.5 + eta)))
        self.iu = rng(lo[0], hi[0], eff_dist)
        self.iv = rng(lo[1], hi[1], eff_dist)
        self.iw = rng(lo[2], hi[2], ws_dist)
        self.grid = np.zeros((N, N), np.complex64)
        self.grid.fill(0)            # first touch outside the timed calls

    def planes(self):
        return list(range(self.iw[0], self.iw[1] + 1))

    def grid_towers(self, iw, task_stride=1, task_offset=0):
        """Sub-grid towers of one w-stack plane into self.grid; returns
        (visibilities gridded, non-empty tasks gridded, present)."""
        L = lib()
        p = lambda a: a.ctypes.data
        sup, os_, wsup, wos = self.kw
        tasks = np.zeros(2, np.int64)
        n = L.port_grid_plane(
            self.R, self.C, p(self.uvw), p(self.vis), self.f0, self.df,
            self.N, self.S, self.theta, self.w_step, sup, os_, wsup, wos,
            p(self.uv_kernel), p(self.w_kernel), p(self.w_pattern),
            self.frac, self.H, iw, self.iu[0], self.iu[1], self.iv[0],
            self.iv[1], p(self.grid), task_stride, task_offset, p(tasks))
        if n < 0:
            raise ValueError("port_grid_plane: bad size")
        return int(n), int(tasks[0]), int(tasks[1])

    def finish_plane(self, iw, image):
        """Plane FFT, grid correction, image += (float32, in place)."""
        L = lib()
        p = lambda a: a.ctypes.data
        assert image.dtype == np.float32 and image.flags.c_contiguous
        if L.port_finish_plane(self.N, p(self.grid), p(image), self.theta,
                               self.w_step, 0.0, 0.0, int(iw * self.H),
                               p(self.pswf_lm), p(self.leg), len(self.leg),
                               self.c_n):
            raise ValueError("port_finish_plane: N must be a power of two")

    def grid_plane(self, iw, image):
        """One w-stack plane into image (N x N float32, +=); returns the
        number of visibilities gridded."""
        n = self.grid_towers(iw)[0]
        if n:
            self.finish_plane(iw, image)
        return n


def grid_all(vis, f0, df, uvw, S, theta, w_step, support, oversampling,
             w_support, w_oversampling, subgrid_frac, H, image):
    """The whole call (image overwritten, float32); returns vis gridded."""
    plan = Plan(vis, f0, df, uvw, image.shape[0], S, theta, w_step, support,
                oversampling, w_support, w_oversampling, subgrid_frac, H)
    image[...] = 0
    return sum(plan.grid_plane(iw, image) for iw in plan.planes())
