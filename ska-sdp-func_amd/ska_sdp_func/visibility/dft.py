"""Point-source DFT prediction of visibilities (MI355X HIP implementation).

Mirrors src/ska_sdp_func/visibility/dft.py of ska-sdp-func 1.2.2: same
function names, arguments and in-place semantics. Arrays may be numpy
(staged through the GPU by the library), torch tensors on a ROCm device or
cupy arrays, all in one location. source_directions [components, 3] and
uvw float64, source_fluxes [components, channels, pols] complex128, vis
[times, baselines, channels, pols] complex128 or complex64.
"""
import ctypes

from ..utility import Lib, Mem

Lib.wrap_func(
    "sdp_dft_point_v00",
    restype=None,
    argtypes=[
        Mem.handle_type(),
        Mem.handle_type(),
        Mem.handle_type(),
        Mem.handle_type(),
    ],
    check_errcode=True,
)

Lib.wrap_func(
    "sdp_dft_point_v01",
    restype=None,
    argtypes=[
        Mem.handle_type(),
        Mem.handle_type(),
        Mem.handle_type(),
        ctypes.c_double,
        ctypes.c_double,
        Mem.handle_type(),
    ],
    check_errcode=True,
)


def dft_point_v00(source_directions, source_fluxes, uvw_lambda, vis):
    """vis[t, b, c, p] = sum_s flux[s, c, p] exp(-2 pi i (l u + m v + n w))
    with uvw_lambda [times, baselines, channels, 3] in wavelengths
    (reference sdp_dft.cpp:24-98). vis is overwritten."""
    Lib.sdp_dft_point_v00(
        Mem(source_directions), Mem(source_fluxes), Mem(uvw_lambda), Mem(vis)
    )


def dft_point_v01(source_directions, source_fluxes, uvw, channel_start_hz,
                  channel_step_hz, vis):
    """As dft_point_v00 with uvw [times, baselines, 3] in metres, scaled per
    channel by (channel_start_hz + c channel_step_hz) / c0 (reference
    sdp_dft.cpp:253-336). vis is overwritten."""
    Lib.sdp_dft_point_v01(
        Mem(source_directions),
        Mem(source_fluxes),
        Mem(uvw),
        channel_start_hz,
        channel_step_hz,
        Mem(vis),
    )
