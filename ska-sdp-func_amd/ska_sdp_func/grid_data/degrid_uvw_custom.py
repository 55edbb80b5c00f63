"""Degridding with caller-supplied kernels (MI355X HIP implementation).

Mirrors src/ska_sdp_func/grid_data/degrid_uvw_custom.py of ska-sdp-func
1.2.2: same function name, arguments and in-place semantics on vis. Arrays
may be numpy (staged through the GPU by the library), torch tensors on a
ROCm device or cupy arrays; double precision only, as the reference.
"""
import ctypes

from ..utility import Lib, Mem

Lib.wrap_func(
    "sdp_degrid_uvw_custom",
    restype=None,
    argtypes=[
        Mem.handle_type(),
        Mem.handle_type(),
        Mem.handle_type(),
        Mem.handle_type(),
        ctypes.c_double,
        ctypes.c_double,
        ctypes.c_double,
        ctypes.c_double,
        ctypes.c_int32,
        Mem.handle_type(),
    ],
    check_errcode=True,
)


def degrid_uvw_custom(grid, uvw, uv_kernel, w_kernel, theta, wstep,
                      channel_start_hz, channel_step_hz, conjugate, vis):
    """Degrid visibilities from grid [chan][w][v][u][pol] with the given
    oversampled uv and w kernels ([oversampling][stride]); vis
    [time][baseline][chan][pol] is written where the kernel footprint lies
    inside the grid (reference sdp_degrid_uvw_custom.cpp:66-180)."""
    Lib.sdp_degrid_uvw_custom(
        Mem(grid),
        Mem(uvw),
        Mem(uv_kernel),
        Mem(w_kernel),
        theta,
        wstep,
        channel_start_hz,
        channel_step_hz,
        int(bool(conjugate)),
        Mem(vis),
    )
