"""Multi-scale CLEAN, Cornwell's algorithm (MI355X HIP implementation).

Mirrors src/ska_sdp_func/clean/ms_clean_cornwell.py of ska-sdp-func 1.2.2:
same function name, arguments and in-place outputs. Images may be numpy
(staged through the GPU by the library), torch tensors on a ROCm device or
cupy arrays, all in one location; scale_list is int32.
"""
import ctypes

from ..utility import Lib, Mem

Lib.wrap_func(
    "sdp_ms_clean_cornwell",
    restype=None,
    argtypes=[
        Mem.handle_type(),
        Mem.handle_type(),
        Mem.handle_type(),
        Mem.handle_type(),
        ctypes.c_double,
        ctypes.c_double,
        ctypes.c_int,
        Mem.handle_type(),
        Mem.handle_type(),
        Mem.handle_type(),
    ],
    check_errcode=True,
)


def ms_clean_cornwell(dirty_img, psf, cbeam_details, scale_list, loop_gain,
                      threshold, cycle_limit, clean_model, residual,
                      skymodel):
    """Multi-scale CLEAN of dirty_img [N, N] with psf [2N, 2N] over the
    scales in scale_list (pixels; reference sdp_ms_clean_cornwell.cpp
    :169-770). Writes the component map, the (scale-0) residual and
    components (*) beam + residual."""
    Lib.sdp_ms_clean_cornwell(
        Mem(dirty_img),
        Mem(psf),
        Mem(cbeam_details),
        Mem(scale_list),
        loop_gain,
        threshold,
        cycle_limit,
        Mem(clean_model),
        Mem(residual),
        Mem(skymodel),
    )
