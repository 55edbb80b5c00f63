"""W-towers sub-grid (de)gridder, MI355X build.

Same class, methods and arguments as the reference
src/ska_sdp_func/grid_data/gridder_wtower_uvw.py:13-575, bound to this
repository's libska_sdp_func. Arrays may be numpy (host: the library stages
them through device memory and still computes on the GPU), or torch / cupy
device arrays. All arrays of one call must share a location.
"""

import ctypes

import numpy

from ..utility import Lib, Mem, StructWrapper


class GridderWtowerUVW(StructWrapper):
    """Plan for (de)gridding sub-grids with w-towers (PSWF kernels)."""

    def __init__(
        self,
        image_size: int,
        subgrid_size: int,
        theta: float,
        w_step: float,
        shear_u: float,
        shear_v: float,
        support: int,
        oversampling: int,
        w_support: int,
        w_oversampling: int,
    ):
        """Create the plan (gridder_wtower_uvw.py:18-60).

        image_size: total image size in pixels; subgrid_size: sub-grid size
        in pixels (even); theta: image size in direction cosines; w_step:
        spacing of w-planes; shear_u / shear_v: shear factors; support /
        oversampling: uv kernel; w_support / w_oversampling: w kernel.
        """
        create_args = (
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
        )
        super().__init__(
            Lib.sdp_gridder_wtower_uvw_create,
            create_args,
            Lib.sdp_gridder_wtower_uvw_free,
        )

    def degrid(
        self,
        subgrid_image,
        subgrid_offset_u: int,
        subgrid_offset_v: int,
        subgrid_offset_w: int,
        freq0_hz: float,
        dfreq_hz: float,
        uvws,
        start_chs,
        end_chs,
        vis,
        start_row: int = -1,
        end_row: int = -1,
    ):
        """Degrid into vis (+=); deprecated form of degrid_subgrid."""
        Lib.sdp_gridder_wtower_uvw_degrid(
            self,
            Mem(subgrid_image),
            subgrid_offset_u,
            subgrid_offset_v,
            subgrid_offset_w,
            freq0_hz,
            dfreq_hz,
            Mem(uvws),
            Mem(start_chs),
            Mem(end_chs),
            Mem(vis),
            start_row,
            end_row,
        )

    def degrid_subgrid(
        self,
        subgrid_image,
        subgrid_offset,
        ch_count: int,
        freq0_hz: float,
        dfreq_hz: float,
        uvws,
        start_chs,
        end_chs,
        vis=None,
        start_row: int = -1,
        end_row: int = -1,
    ):
        """Degrid visibilities; returns a new complex128 array if vis is
        None (gridder_wtower_uvw.py:123-188)."""
        (subgrid_offset_u, subgrid_offset_v, subgrid_offset_w) = subgrid_offset
        return_vis = False
        if vis is None:
            vis = numpy.zeros(
                (uvws.shape[0], ch_count), dtype=numpy.complex128
            )
            return_vis = True
        Lib.sdp_gridder_wtower_uvw_degrid(
            self,
            Mem(subgrid_image),
            subgrid_offset_u,
            subgrid_offset_v,
            subgrid_offset_w,
            freq0_hz,
            dfreq_hz,
            Mem(uvws),
            Mem(start_chs),
            Mem(end_chs),
            Mem(vis),
            start_row,
            end_row,
        )
        if return_vis:
            return vis
        return None

    def degrid_correct(
        self,
        facet,
        facet_offset_l: int,
        facet_offset_m: int,
        w_offset: int = 0,
    ):
        """Degrid correction of a facet, in place; returns the facet."""
        Lib.sdp_gridder_wtower_uvw_degrid_correct(
            self, Mem(facet), facet_offset_l, facet_offset_m, w_offset
        )
        return facet

    def grid(
        self,
        vis,
        uvw,
        start_chs,
        end_chs,
        freq0_hz: float,
        dfreq_hz: float,
        subgrid_image,
        subgrid_offset_u: int,
        subgrid_offset_v: int,
        subgrid_offset_w: int,
        start_row: int = -1,
        end_row: int = -1,
    ):
        """Grid into subgrid_image (+=); deprecated form of grid_subgrid."""
        Lib.sdp_gridder_wtower_uvw_grid(
            self,
            Mem(vis),
            Mem(uvw),
            Mem(start_chs),
            Mem(end_chs),
            freq0_hz,
            dfreq_hz,
            Mem(subgrid_image),
            subgrid_offset_u,
            subgrid_offset_v,
            subgrid_offset_w,
            start_row,
            end_row,
        )

    def grid_subgrid(
        self,
        vis,
        uvw,
        start_chs,
        end_chs,
        ch_count: int,
        freq0_hz: float,
        dfreq_hz: float,
        subgrid_image,
        subgrid_offset,
        start_row: int = -1,
        end_row: int = -1,
    ):
        """Grid visibilities into subgrid_image (+=)
        (gridder_wtower_uvw.py:273-330)."""
        (subgrid_offset_u, subgrid_offset_v, subgrid_offset_w) = subgrid_offset
        if ch_count and vis.shape[1] != ch_count:
            raise RuntimeError("Inconsistent channel dimensions")
        Lib.sdp_gridder_wtower_uvw_grid(
            self,
            Mem(vis),
            Mem(uvw),
            Mem(start_chs),
            Mem(end_chs),
            freq0_hz,
            dfreq_hz,
            Mem(subgrid_image),
            subgrid_offset_u,
            subgrid_offset_v,
            subgrid_offset_w,
            start_row,
            end_row,
        )

    def grid_correct(
        self,
        facet,
        facet_offset_l: int,
        facet_offset_m: int,
        w_offset: int = 0,
    ):
        """Grid correction of a facet, in place; returns the facet."""
        Lib.sdp_gridder_wtower_uvw_grid_correct(
            self, Mem(facet), facet_offset_l, facet_offset_m, w_offset
        )
        return facet

    def num_w_planes(self, gridding: bool = False):
        """w-planes processed so far by degrid (False) or grid (True)."""
        return Lib.sdp_gridder_wtower_uvw_num_w_planes(self, int(gridding))

    @property
    def image_size(self):
        """Image size in pixels."""
        return Lib.sdp_gridder_wtower_uvw_image_size(self)

    @property
    def oversampling(self):
        """Oversampling of the uv kernel."""
        return Lib.sdp_gridder_wtower_uvw_oversampling(self)

    @property
    def shear_u(self):
        """Shear factor in u."""
        return Lib.sdp_gridder_wtower_uvw_shear_u(self)

    @property
    def shear_v(self):
        """Shear factor in v."""
        return Lib.sdp_gridder_wtower_uvw_shear_v(self)

    @property
    def subgrid_size(self):
        """Sub-grid size in pixels."""
        return Lib.sdp_gridder_wtower_uvw_subgrid_size(self)

    @property
    def support(self):
        """Support of the uv kernel."""
        return Lib.sdp_gridder_wtower_uvw_support(self)

    @property
    def theta(self):
        """Image size in direction cosines."""
        return Lib.sdp_gridder_wtower_uvw_theta(self)

    @property
    def w_oversampling(self):
        """Oversampling of the w kernel."""
        return Lib.sdp_gridder_wtower_uvw_w_oversampling(self)

    @property
    def w_step(self):
        """Spacing of w-planes."""
        return Lib.sdp_gridder_wtower_uvw_w_step(self)

    @property
    def w_support(self):
        """Support of the w kernel."""
        return Lib.sdp_gridder_wtower_uvw_w_support(self)


_H = GridderWtowerUVW.handle_type()
_M = Mem.handle_type()
_I = ctypes.c_int
_D = ctypes.c_double
_I64 = ctypes.c_int64

Lib.wrap_func(
    "sdp_gridder_wtower_uvw_create",
    restype=_H,
    argtypes=[_I, _I, _D, _D, _D, _D, _I, _I, _I, _I],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_wtower_uvw_degrid",
    restype=None,
    argtypes=[_H, _M, _I, _I, _I, _D, _D, _M, _M, _M, _M, _I64, _I64],
    check_errcode=True,
)
Lib.wrap_func(
    "sdp_gridder_wtower_uvw_grid",
    restype=None,
    argtypes=[_H, _M, _M, _M, _M, _D, _D, _M, _I, _I, _I, _I64, _I64],
    check_errcode=True,
)
for _name in ("degrid_correct", "grid_correct"):
    Lib.wrap_func(
        f"sdp_gridder_wtower_uvw_{_name}",
        restype=None,
        argtypes=[_H, _M, _I, _I, _I],
        check_errcode=True,
    )
Lib.wrap_func("sdp_gridder_wtower_uvw_free", restype=None, argtypes=[_H])
Lib.wrap_func(
    "sdp_gridder_wtower_uvw_num_w_planes", restype=_I, argtypes=[_H, _I]
)
for _name in ("image_size", "oversampling", "subgrid_size", "support",
              "w_oversampling", "w_support"):
    Lib.wrap_func(f"sdp_gridder_wtower_uvw_{_name}", restype=_I,
                  argtypes=[_H])
for _name in ("shear_u", "shear_v", "theta", "w_step"):
    Lib.wrap_func(f"sdp_gridder_wtower_uvw_{_name}", restype=_D,
                  argtypes=[_H])
