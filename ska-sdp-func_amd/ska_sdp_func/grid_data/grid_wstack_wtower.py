"""W-stacking with w-towers over a whole image, MI355X build.

Same functions and arguments as the reference
src/ska_sdp_func/grid_data/grid_wstack_wtower.py:12-196. num_threads is
accepted and ignored (the work runs on the GPU). The *_planes variants are
an extension that processes a subset of the w-stack planes, for sharding
planes across GPUs (one process per GPU; the outputs of all shards sum to
the full result).
"""

import ctypes
from typing import Optional

from ..utility import Lib, Mem


def wstack_wtower_degrid_all(
    image,
    freq0_hz: float,
    dfreq_hz: float,
    uvw,
    subgrid_size: int,
    theta: float,
    w_step: float,
    shear_u: float,
    shear_v: float,
    support: int,
    oversampling: int,
    w_support: int,
    w_oversampling: int,
    subgrid_frac: float,
    w_tower_height: float,
    verbosity: int,
    vis,
    num_threads: Optional[int] = None,
):
    """Degrid visibilities (vis is overwritten) from the image
    (grid_wstack_wtower.py:12-75)."""
    if not num_threads:
        num_threads = 0
    Lib.sdp_grid_wstack_wtower_degrid_all(
        Mem(image), freq0_hz, dfreq_hz, Mem(uvw), subgrid_size, theta,
        w_step, shear_u, shear_v, support, oversampling, w_support,
        w_oversampling, subgrid_frac, w_tower_height, verbosity, Mem(vis),
        num_threads,
    )


def wstack_wtower_grid_all(
    vis,
    freq0_hz: float,
    dfreq_hz: float,
    uvw,
    subgrid_size: int,
    theta: float,
    w_step: float,
    shear_u: float,
    shear_v: float,
    support: int,
    oversampling: int,
    w_support: int,
    w_oversampling: int,
    subgrid_frac: float,
    w_tower_height: float,
    verbosity: int,
    image,
    num_threads: Optional[int] = None,
):
    """Grid visibilities into the image (overwritten)
    (grid_wstack_wtower.py:78-143)."""
    if not num_threads:
        num_threads = 0
    Lib.sdp_grid_wstack_wtower_grid_all(
        Mem(vis), freq0_hz, dfreq_hz, Mem(uvw), subgrid_size, theta,
        w_step, shear_u, shear_v, support, oversampling, w_support,
        w_oversampling, subgrid_frac, w_tower_height, verbosity, Mem(image),
        num_threads,
    )


def wstack_wtower_degrid_planes(image, freq0_hz, dfreq_hz, uvw,
                                subgrid_size, theta, w_step, shear_u,
                                shear_v, support, oversampling, w_support,
                                w_oversampling, subgrid_frac,
                                w_tower_height, verbosity, vis,
                                plane_offset: int = 0,
                                plane_stride: int = 1):
    """degrid_all restricted to w-stack planes with
    (iw - min_iw) % plane_stride == plane_offset."""
    Lib.sdp_grid_wstack_wtower_degrid_planes(
        Mem(image), freq0_hz, dfreq_hz, Mem(uvw), subgrid_size, theta,
        w_step, shear_u, shear_v, support, oversampling, w_support,
        w_oversampling, subgrid_frac, w_tower_height, verbosity, Mem(vis),
        plane_offset, plane_stride,
    )


def wstack_wtower_grid_planes(vis, freq0_hz, dfreq_hz, uvw, subgrid_size,
                              theta, w_step, shear_u, shear_v, support,
                              oversampling, w_support, w_oversampling,
                              subgrid_frac, w_tower_height, verbosity, image,
                              plane_offset: int = 0, plane_stride: int = 1):
    """grid_all restricted to w-stack planes with
    (iw - min_iw) % plane_stride == plane_offset."""
    Lib.sdp_grid_wstack_wtower_grid_planes(
        Mem(vis), freq0_hz, dfreq_hz, Mem(uvw), subgrid_size, theta,
        w_step, shear_u, shear_v, support, oversampling, w_support,
        w_oversampling, subgrid_frac, w_tower_height, verbosity, Mem(image),
        plane_offset, plane_stride,
    )


def wstack_wtower_grid_plane_set(vis, freq0_hz, dfreq_hz, uvw, subgrid_size,
                                 theta, w_step, shear_u, shear_v, support,
                                 oversampling, w_support, w_oversampling,
                                 subgrid_frac, w_tower_height, verbosity,
                                 image, plane_first: int, plane_mask):
    """grid_all restricted to the w-stack planes iw (the reference's plane
    index) with plane_mask[iw - plane_first] != 0; plane_mask: 1-D int32
    array (numpy or torch, host or device)."""
    Lib.sdp_grid_wstack_wtower_grid_plane_set(
        Mem(vis), freq0_hz, dfreq_hz, Mem(uvw), subgrid_size, theta,
        w_step, shear_u, shear_v, support, oversampling, w_support,
        w_oversampling, subgrid_frac, w_tower_height, verbosity, Mem(image),
        int(plane_first), Mem(plane_mask),
    )


def wstack_wtower_degrid_plane_set(image, freq0_hz, dfreq_hz, uvw,
                                   subgrid_size, theta, w_step, shear_u,
                                   shear_v, support, oversampling, w_support,
                                   w_oversampling, subgrid_frac,
                                   w_tower_height, verbosity, vis,
                                   plane_first: int, plane_mask):
    """degrid_all restricted to the planes of plane_mask (see
    wstack_wtower_grid_plane_set)."""
    Lib.sdp_grid_wstack_wtower_degrid_plane_set(
        Mem(image), freq0_hz, dfreq_hz, Mem(uvw), subgrid_size, theta,
        w_step, shear_u, shear_v, support, oversampling, w_support,
        w_oversampling, subgrid_frac, w_tower_height, verbosity, Mem(vis),
        int(plane_first), Mem(plane_mask),
    )


def wstack_wtower_enable_timing(enable: bool = True):
    """Switch HIP-event timing of the fused tower kernels on (resetting
    the totals) or off."""
    Lib.sdp_grid_wstack_wtower_enable_timing(int(enable))


def wstack_wtower_get_timing():
    """Totals since enable_timing(True): dict with kernel_ms, launches,
    vis, layers, subgrid_size, kind ("grid" / "degrid"); None when off."""
    out = (ctypes.c_double * 6)()
    n = Lib.sdp_grid_wstack_wtower_get_timing(out, 6)
    if n < 6:
        return None
    return {"kernel_ms": out[0], "launches": int(out[1]), "vis": int(out[2]),
            "layers": int(out[3]), "subgrid_size": int(out[4]),
            "kind": "degrid" if out[5] else "grid"}


_M = Mem.handle_type()
_I = ctypes.c_int
_D = ctypes.c_double
_COMMON = [_D, _D, _M, _I, _D, _D, _D, _D, _I, _I, _I, _I, _D, _D, _I, _M]

for _name in ("degrid_all", "grid_all"):
    Lib.wrap_func(f"sdp_grid_wstack_wtower_{_name}", restype=None,
                  argtypes=[_M] + _COMMON + [_I], check_errcode=True)
for _name in ("degrid_planes", "grid_planes"):
    Lib.wrap_func(f"sdp_grid_wstack_wtower_{_name}", restype=None,
                  argtypes=[_M] + _COMMON + [_I, _I], check_errcode=True)
for _name in ("degrid_plane_set", "grid_plane_set"):
    Lib.wrap_func(f"sdp_grid_wstack_wtower_{_name}", restype=None,
                  argtypes=[_M] + _COMMON + [ctypes.c_int64, _M],
                  check_errcode=True)
Lib.wrap_func("sdp_grid_wstack_wtower_enable_timing", restype=None,
              argtypes=[_I])
Lib.wrap_func("sdp_grid_wstack_wtower_get_timing", restype=_I,
              argtypes=[ctypes.POINTER(_D), _I])
