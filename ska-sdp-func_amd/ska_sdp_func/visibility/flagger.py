"""Dynamic-threshold RFI flagger (MI355X HIP implementation).

Mirrors src/ska_sdp_func/visibility/flagger.py of ska-sdp-func 1.2.2:
same function name, arguments and in-place semantics. Arrays may be numpy
(staged through the GPU by the library), torch tensors on a ROCm device or
cupy arrays; vis is [time, baseline, channel, pol] complex64/complex128 and
flags the int32 array of the same shape (flags are only set, never
cleared).
"""
import ctypes

from ..utility import Lib, Mem

Lib.wrap_func(
    "sdp_flagger_dynamic_threshold",
    restype=None,
    argtypes=[
        Mem.handle_type(),
        Mem.handle_type(),
        ctypes.c_double,
        ctypes.c_double,
        ctypes.c_double,
        ctypes.c_double,
        ctypes.c_int,
        ctypes.c_int,
        ctypes.c_int,
    ],
    check_errcode=True,
)


def flagger_dynamic_threshold(
    vis,
    flags,
    alpha: float,
    threshold_magnitudes: float,
    threshold_variations: float,
    threshold_broadband: float,
    sampling_step: int,
    window: int,
    window_median_history: int,
):
    """Flag unusually large magnitudes, unusually fluctuating magnitudes and
    broadband jumps of the per-time-step median (reference
    sdp_flagger.cpp:125-339). See the reference docstring for the meaning of
    the parameters."""
    Lib.sdp_flagger_dynamic_threshold(
        Mem(vis),
        Mem(flags),
        alpha,
        threshold_magnitudes,
        threshold_variations,
        threshold_broadband,
        sampling_step,
        window,
        window_median_history,
    )
