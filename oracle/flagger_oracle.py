"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the dynamic-threshold flagger.

Wraps oracle/flagger_oracle.c, a restatement of
  sdp_flagger_dynamic_threshold  src/ska-sdp-func/visibility/sdp_flagger.cpp:125-428
(ska-sdp-func 1.2.2). Used only by tests/, as the checker of the HIP flagger.

Parity status: building / running the reference flagger here was denied
("Denied"); the restatement is pinned by the reference's own
known-answer test (tests/visibility/test_flagger.py:11-65), reproduced in
tests/test_flagger_oracle.py.
"""
import ctypes
import os
import subprocess

import numpy as np

from . import _cc

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def build(force=False):
    """Compile oracle/flagger_oracle.c (gcc, OpenMP) (oracle/_cc.py)."""
    return _cc.shared("flagger_oracle.c", "libflagger_oracle.so",
                      ["-O2", "-fopenmp", "-fno-fast-math", "-ffp-contract=off"],
                      force)


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
        P = ctypes.c_void_p
        i32, i64, f64 = ctypes.c_int, ctypes.c_int64, ctypes.c_double
        _lib.oracle_flagger.argtypes = [P, i32, P, f64, f64, f64, f64, i32,
                                        i32, i32, i64, i64, i32, i32]
        _lib.oracle_flagger.restype = None
        _lib.oracle_flagger_set_threads.argtypes = [i32]
        _lib.oracle_flagger_set_threads.restype = i32
        _lib.oracle_cabs_f32.argtypes = [P, i64, P]
        _lib.oracle_cabs_f64.argtypes = [P, i64, P]
    return _lib


def flagger_dynamic_threshold(vis, flags, alpha, threshold_magnitudes,
                              threshold_variations, threshold_broadband,
                              sampling_step, window, window_median_history):
    """Same arguments and in-place semantics as the reference Python
    function (src/ska_sdp_func/visibility/flagger.py); numpy arrays only."""
    assert vis.ndim == 4 and flags.shape == vis.shape
    assert vis.dtype in (np.complex64, np.complex128)
    assert flags.dtype == np.int32
    assert vis.flags.c_contiguous and flags.flags.c_contiguous
    T, B, C, P = vis.shape
    lib().oracle_flagger(vis.ctypes.data, int(vis.dtype == np.complex128),
                         flags.ctypes.data, float(alpha),
                         float(threshold_magnitudes),
                         float(threshold_variations),
                         float(threshold_broadband), int(sampling_step),
                         int(window), int(window_median_history), T, B, C, P)
    return flags


def cabs(vis):
    """|v| as glibc cabsf / cabs give it (float64 array)."""
    v = np.ascontiguousarray(vis)
    out = np.empty(v.shape, np.float64)
    fn = (lib().oracle_cabs_f64 if v.dtype == np.complex128
          else lib().oracle_cabs_f32)
    fn(v.ctypes.data, v.size, out.ctypes.data)
    return out
