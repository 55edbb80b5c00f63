"""Hogbom CLEAN (MI355X HIP implementation).

Mirrors src/ska_sdp_func/clean/hogbom_clean.py of ska-sdp-func 1.2.2: same
function name, arguments and in-place outputs. Images may be numpy (staged
through the GPU by the library), torch tensors on a ROCm device or cupy
arrays, all in one location; cbeam_details may live anywhere.
"""
import ctypes

from ..utility import Lib, Mem

Lib.wrap_func(
    "sdp_hogbom_clean",
    restype=None,
    argtypes=[
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


def hogbom_clean(dirty_img, psf, cbeam_details, loop_gain, threshold,
                 cycle_limit, clean_model, residual, skymodel):
    """Hogbom CLEAN of dirty_img [N, N] with psf [2N, 2N].

    cbeam_details = [BMAJ sigma, BMIN sigma, THETA degrees, SIZE] of the
    Gaussian CLEAN beam. Writes the component map to clean_model, the
    residual to residual and components (*) beam + residual to skymodel
    (reference sdp_hogbom_clean.cpp:113-278). Stops after cycle_limit
    cycles or when the residual peak falls below threshold.
    """
    Lib.sdp_hogbom_clean(
        Mem(dirty_img),
        Mem(psf),
        Mem(cbeam_details),
        loop_gain,
        threshold,
        cycle_limit,
        Mem(clean_model),
        Mem(residual),
        Mem(skymodel),
    )
