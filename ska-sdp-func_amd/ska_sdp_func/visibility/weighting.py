"""Visibility weighting, uniform and Briggs (MI355X HIP implementation).

Mirrors src/ska_sdp_func/visibility/weighting.py of ska-sdp-func 1.2.2:
same function names, arguments and in-place semantics. Arrays may be numpy
(staged through the GPU by the library), torch tensors on a ROCm device or
cupy arrays. uvw is [time, baseline, 3] float64, freq_hz [channel] float64,
grid_uv [grid, grid, pol] and the weights [time, baseline, channel, pol],
all float64 or all float32 (grid and weights).
"""
import ctypes

import numpy

from ..utility import Lib, Mem

Lib.wrap_func(
    "sdp_weighting_briggs",
    restype=None,
    argtypes=[
        Mem.handle_type(),
        Mem.handle_type(),
        ctypes.c_double,
        ctypes.c_double,
        Mem.handle_type(),
        Mem.handle_type(),
        Mem.handle_type(),
    ],
    check_errcode=True,
)

Lib.wrap_func(
    "sdp_weighting_uniform",
    restype=None,
    argtypes=[
        Mem.handle_type(),
        Mem.handle_type(),
        ctypes.c_double,
        Mem.handle_type(),
        Mem.handle_type(),
        Mem.handle_type(),
    ],
    check_errcode=True,
)


def get_uv_range(uvw, freq_hz):
    """Largest |u| over all baselines (only the u coordinate, as the
    reference's weighting.py:41-58) times the last frequency over c, i.e.
    max_abs_uv in wavelengths."""
    if hasattr(uvw, "detach"):   # torch tensor
        u = uvw[:, :, 0:1].abs().max().item()
        f = float(freq_hz[-1])
    else:
        u = float(numpy.amax(numpy.abs(uvw[:, :, 0:1])))
        f = float(freq_hz[-1])
    return u * f / 299792458.0


def briggs_weights(uvw, freq_hz, max_abs_uv, robust_param, grid_uv,
                   input_weights, output_weights):
    """Robust (Briggs) weights: grid_uv accumulates the input weights per
    uv cell; output = input / (1 + R grid), R = (5 10^-robust)^2 /
    (sum grid^2 / sum grid) over the visibilities (reference
    sdp_weighting.cpp:143-154)."""
    Lib.sdp_weighting_briggs(
        Mem(uvw),
        Mem(freq_hz),
        max_abs_uv,
        robust_param,
        Mem(grid_uv),
        Mem(input_weights),
        Mem(output_weights),
    )


def uniform_weights(uvw, freq_hz, max_abs_uv, grid_uv, input_weights,
                    output_weights):
    """Uniform weights: grid_uv accumulates the input weights per uv cell;
    output = 1 / grid (reference sdp_weighting.cpp:158-217)."""
    Lib.sdp_weighting_uniform(
        Mem(uvw),
        Mem(freq_hz),
        max_abs_uv,
        Mem(grid_uv),
        Mem(input_weights),
        Mem(output_weights),
    )
