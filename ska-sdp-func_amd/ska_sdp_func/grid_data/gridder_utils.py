"""Utility functions of the w-towers gridders, MI355X build.

Same functions and arguments as the reference
src/ska_sdp_func/grid_data/gridder_utils.py:13-541. Array operations run
on the GPU (host arrays are staged through device memory); the kernel-table
generators fill host arrays, as in the reference.
"""

import ctypes
from typing import Optional

from ..utility import Lib, Mem
from .gridder_wtower_uvw import GridderWtowerUVW


def clamp_channels_single(
    uvws,
    dim: int,
    freq0_hz: float,
    dfreq_hz: float,
    start_ch_in,
    end_ch_in,
    min_u: float,
    max_u: float,
    start_ch_out,
    end_ch_out,
    start_row: int = -1,
    end_row: int = -1,
):
    """Restrict channel ranges so that min_u <= uvws[:, dim] * f / c < max_u
    (gridder_utils.py:13-61)."""
    Lib.sdp_gridder_clamp_channels_single(
        Mem(uvws),
        dim,
        freq0_hz,
        dfreq_hz,
        Mem(start_ch_in),
        Mem(end_ch_in),
        min_u,
        max_u,
        Mem(start_ch_out),
        Mem(end_ch_out),
        start_row,
        end_row,
    )


def clamp_channels_uv(
    uvws,
    freq0_hz: float,
    dfreq_hz: float,
    start_ch_in,
    end_ch_in,
    min_u: float,
    max_u: float,
    min_v: float,
    max_v: float,
    start_ch_out,
    end_ch_out,
    start_row: int = -1,
    end_row: int = -1,
):
    """Restrict channel ranges in u and v (gridder_utils.py:64-115)."""
    Lib.sdp_gridder_clamp_channels_uv(
        Mem(uvws),
        freq0_hz,
        dfreq_hz,
        Mem(start_ch_in),
        Mem(end_ch_in),
        min_u,
        max_u,
        min_v,
        max_v,
        Mem(start_ch_out),
        Mem(end_ch_out),
        start_row,
        end_row,
    )


def determine_max_w_tower_height(
    subgrid_size: int,
    theta: float,
    fov: float,
    w_step: float,
    support: int,
    oversampling: int,
    w_support: int,
    w_oversampling: int,
    image_size: Optional[int] = None,
    shear_u: float = 0.0,
    shear_v: float = 0.0,
    subgrid_frac: float = 2.0 / 3.0,
    num_samples: int = 3,
    target_err: Optional[float] = None,
) -> float:
    """Maximum w-tower height (units of w_step) by trial and error
    (gridder_utils.py:118-178)."""
    if not image_size:
        image_size = 2 * subgrid_size
    if not target_err:
        target_err = 0.0
    return Lib.sdp_gridder_determine_max_w_tower_height(
        image_size,
        subgrid_size,
        theta,
        w_step,
        shear_u,
        shear_v,
        support,
        oversampling,
        w_support,
        w_oversampling,
        fov,
        subgrid_frac,
        num_samples,
        target_err,
    )


def determine_w_step(
    theta: float,
    fov: float,
    shear_u: float = 0.0,
    shear_v: float = 0.0,
    x_0: Optional[float] = None,
) -> float:
    """A w_step adequate for the field of view (gridder_utils.py:181-203)."""
    if not x_0:
        x_0 = 0.0
    return float(
        Lib.sdp_gridder_determine_w_step(theta, fov, shear_u, shear_v, x_0)
    )


def find_max_w_tower_height(
    grid_kernel: GridderWtowerUVW,
    fov: float,
    subgrid_frac: float = 2.0 / 3.0,
    num_samples: int = 3,
    target_err: Optional[float] = None,
):
    """determine_max_w_tower_height for an existing gridder
    (gridder_utils.py:206-244)."""
    if not target_err:
        target_err = 0.0
    return Lib.sdp_gridder_determine_max_w_tower_height(
        grid_kernel.image_size,
        grid_kernel.subgrid_size,
        grid_kernel.theta,
        grid_kernel.w_step,
        grid_kernel.shear_u,
        grid_kernel.shear_v,
        grid_kernel.support,
        grid_kernel.oversampling,
        grid_kernel.w_support,
        grid_kernel.w_oversampling,
        fov,
        subgrid_frac,
        num_samples,
        target_err,
    )


def make_kernel(window, kernel):
    """Oversampled kernel [oversampling + 1, support] from an image-space
    window [support] (host arrays)."""
    Lib.sdp_gridder_make_kernel(Mem(window), Mem(kernel))


def make_pswf_kernel(support: int, kernel):
    """PSWF kernel [oversampling + 1, vr_size] (host array)."""
    Lib.sdp_gridder_make_pswf_kernel(support, Mem(kernel))


def make_w_pattern(
    subgrid_size: int,
    theta: float,
    shear_u: float,
    shear_v: float,
    w_step: float,
    w_pattern,
):
    """exp(2 pi i w_step n(l, m)) over the sub-grid (complex128 host)."""
    Lib.sdp_gridder_make_w_pattern(
        subgrid_size, theta, shear_u, shear_v, w_step, Mem(w_pattern)
    )


def rms_diff(array_a, array_b):
    """RMS of a - b for two 2-D arrays of the same shape."""
    return Lib.sdp_gridder_rms_diff(Mem(array_a), Mem(array_b))


def subgrid_add(grid, offset_u: int, offset_v: int, subgrid,
                factor: float = 1.0):
    """grid (periodic) += factor * subgrid placed at -offset."""
    Lib.sdp_gridder_subgrid_add(
        Mem(grid), offset_u, offset_v, Mem(subgrid), factor
    )


def subgrid_cut_out(grid, offset_u: int, offset_v: int, subgrid):
    """subgrid = grid (periodic) at offset."""
    Lib.sdp_gridder_subgrid_cut_out(
        Mem(grid), offset_u, offset_v, Mem(subgrid)
    )


def uvw_bounds_all(uvws, freq0_hz: float, dfreq_hz: float, start_ch, end_ch):
    """(uvw_min, uvw_max) of the selected channels, scaled to wavelengths."""
    min_uvw = (ctypes.c_double * 3)(0.0, 0.0, 0.0)
    max_uvw = (ctypes.c_double * 3)(0.0, 0.0, 0.0)
    Lib.sdp_gridder_uvw_bounds_all(
        Mem(uvws),
        freq0_hz,
        dfreq_hz,
        Mem(start_ch),
        Mem(end_ch),
        min_uvw,
        max_uvw,
    )
    return (min_uvw, max_uvw)


_M = Mem.handle_type()
_I = ctypes.c_int
_D = ctypes.c_double
_I64 = ctypes.c_int64


def _opt(x):
    return Mem(x) if x is not None else None


def count_nonzero_pixels(image) -> int:
    """Number of non-zero pixels (sdp_gridder_count_nonzero_pixels,
    reference sdp_gridder_utils.h:54)."""
    return int(Lib.sdp_gridder_count_nonzero_pixels(Mem(image)))


def dft(uvws, start_chs, end_chs, flux, lmn, subgrid_offset_u: int,
        subgrid_offset_v: int, subgrid_offset_w: int, theta: float,
        w_step: float, freq0_hz: float, dfreq_hz: float, vis):
    """vis += direct Fourier sum of point sources (sdp_gridder_dft,
    reference sdp_gridder_utils.h:99). start_chs / end_chs may be None."""
    Lib.sdp_gridder_dft(Mem(uvws), _opt(start_chs), _opt(end_chs),
                        Mem(flux), Mem(lmn), subgrid_offset_u,
                        subgrid_offset_v, subgrid_offset_w, theta, w_step,
                        freq0_hz, dfreq_hz, Mem(vis))


def idft(uvws, vis, start_chs, end_chs, lmn, image_taper_1d,
         subgrid_offset_u: int, subgrid_offset_v: int, subgrid_offset_w: int,
         theta: float, w_step: float, freq0_hz: float, dfreq_hz: float,
         image):
    """image += direct inverse Fourier sum of the visibilities at the
    pixel directions lmn (sdp_gridder_idft, reference
    sdp_gridder_utils.h:140)."""
    Lib.sdp_gridder_idft(Mem(uvws), Mem(vis), _opt(start_chs), _opt(end_chs),
                         Mem(lmn), _opt(image_taper_1d), subgrid_offset_u,
                         subgrid_offset_v, subgrid_offset_w, theta, w_step,
                         freq0_hz, dfreq_hz, Mem(image))


def image_to_flmn(image, theta: float, shear_u: float, shear_v: float,
                  image_taper_1d, flux, lmn):
    """Pixel direction cosines (and non-zero pixel fluxes when flux is
    given) into host arrays (sdp_gridder_image_to_flmn, reference
    sdp_gridder_utils.h:181)."""
    Lib.sdp_gridder_image_to_flmn(Mem(image), theta, shear_u, shear_v,
                                  _opt(image_taper_1d), _opt(flux), Mem(lmn))


def residual(array_a, array_b, out):
    """out = a - b, out a host array (sdp_gridder_residual, reference
    sdp_gridder_utils.h:260)."""
    Lib.sdp_gridder_residual(Mem(array_a), Mem(array_b), Mem(out))


def grid_correct_pswf(image_size: int, theta: float, w_step: float,
                      shear_u: float, shear_v: float, support: int,
                      w_support: int, facet, facet_offset_l: int,
                      facet_offset_m: int):
    """facet /= pswf(l) pswf(m) pswf_n(n) (sdp_gridder_grid_correct_pswf,
    reference sdp_gridder_grid_correct.h:31)."""
    Lib.sdp_gridder_grid_correct_pswf(image_size, theta, w_step, shear_u,
                                      shear_v, support, w_support,
                                      Mem(facet), facet_offset_l,
                                      facet_offset_m)


def grid_correct_w_stack(image_size: int, theta: float, w_step: float,
                         shear_u: float, shear_v: float, facet,
                         facet_offset_l: int, facet_offset_m: int,
                         w_offset: int, inverse: bool):
    """facet *= exp(-+2 pi i w_step n w_offset)
    (sdp_gridder_grid_correct_w_stack, reference
    sdp_gridder_grid_correct.h:60)."""
    Lib.sdp_gridder_grid_correct_w_stack(image_size, theta, w_step, shear_u,
                                         shear_v, Mem(facet),
                                         facet_offset_l, facet_offset_m,
                                         w_offset, int(bool(inverse)))


Lib.wrap_func(
    "sdp_gridder_clamp_channels_single",
    restype=None,
    argtypes=[_M, _I, _D, _D, _M, _M, _D, _D, _M, _M, _I64, _I64],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_clamp_channels_uv",
    restype=None,
    argtypes=[_M, _D, _D, _M, _M, _D, _D, _D, _D, _M, _M, _I64, _I64],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_determine_max_w_tower_height",
    restype=_D,
    argtypes=[_I, _I, _D, _D, _D, _D, _I, _I, _I, _I, _D, _D, _I, _D],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_determine_w_step",
    restype=_D,
    argtypes=[_D, _D, _D, _D, _D],
)
Lib.wrap_func(
    "sdp_gridder_make_kernel",
    restype=None,
    argtypes=[_M, _M],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_make_pswf_kernel",
    restype=None,
    argtypes=[_I, _M],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_make_w_pattern",
    restype=None,
    argtypes=[_I, _D, _D, _D, _D, _M],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_rms_diff",
    restype=_D,
    argtypes=[_M, _M],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_subgrid_add",
    restype=None,
    argtypes=[_M, _I, _I, _M, _D],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_subgrid_cut_out",
    restype=None,
    argtypes=[_M, _I, _I, _M],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_uvw_bounds_all",
    restype=None,
    argtypes=[_M, _D, _D, _M, _M, ctypes.POINTER(ctypes.c_double),
              ctypes.POINTER(ctypes.c_double)],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_count_nonzero_pixels",
    restype=ctypes.c_int64,
    argtypes=[_M],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_dft",
    restype=None,
    argtypes=[_M, _M, _M, _M, _M, _I, _I, _I, _D, _D, _D, _D, _M],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_idft",
    restype=None,
    argtypes=[_M, _M, _M, _M, _M, _M, _I, _I, _I, _D, _D, _D, _D, _M],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_image_to_flmn",
    restype=None,
    argtypes=[_M, _D, _D, _D, _M, _M, _M],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_residual",
    restype=None,
    argtypes=[_M, _M, _M],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_grid_correct_pswf",
    restype=None,
    argtypes=[_I, _D, _D, _D, _D, _I, _I, _M, _I, _I],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_grid_correct_w_stack",
    restype=None,
    argtypes=[_I, _D, _D, _D, _D, _M, _I, _I, _I, _I],
    check_errcode=True,
)
