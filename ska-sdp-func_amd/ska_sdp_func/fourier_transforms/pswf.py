"""Prolate spheroidal wave functions (C ABI sdp_pswf.h of the reference,
src/ska-sdp-func/fourier_transforms/sdp_pswf.h:27-137; the reference has
no Python binding for it, this one is an extension of the MI355X build)."""

import ctypes

from ..utility import Lib, Mem, StructWrapper


def generate_pswf(m: int, c: float, out):
    """Fill the 1-D host array out with S_mm(c, x) at x = 2 (i - n/2) / n
    (element 0 is 0), sdp_generate_pswf."""
    Lib.sdp_generate_pswf(m, c, Mem(out))


class Pswf(StructWrapper):
    """S_mm(c, x) (sdp_pswf_create / sdp_pswf_evaluate)."""

    def __init__(self, m: int, c: float):
        super().__init__(Lib.sdp_pswf_create, (m, c), Lib.sdp_pswf_free)

    def evaluate(self, x: float) -> float:
        """S(|x|) for |x| < 1, else 0."""
        return Lib.sdp_pswf_evaluate(self, x)

    @property
    def c(self) -> float:
        return Lib.sdp_pswf_par_c(self)

    @property
    def m(self) -> int:
        return int(Lib.sdp_pswf_par_m(self))

    def generate(self, out=None, size: int = 0, end_correction=False):
        """Fill out (1-D host array), or the plan's own table of size
        points (sdp_pswf_generate)."""
        Lib.sdp_pswf_generate(self, Mem(out) if out is not None else None,
                              size, int(bool(end_correction)))


_P = Pswf.handle_type()
Lib.wrap_func("sdp_generate_pswf", restype=None,
              argtypes=[ctypes.c_int, ctypes.c_double, Mem.handle_type()],
              check_errcode=True)
Lib.wrap_func("sdp_pswf_create", restype=_P,
              argtypes=[ctypes.c_int, ctypes.c_double])
Lib.wrap_func("sdp_pswf_free", restype=None, argtypes=[_P])
Lib.wrap_func("sdp_pswf_evaluate", restype=ctypes.c_double,
              argtypes=[_P, ctypes.c_double])
Lib.wrap_func("sdp_pswf_par_c", restype=ctypes.c_double, argtypes=[_P])
Lib.wrap_func("sdp_pswf_par_m", restype=ctypes.c_double, argtypes=[_P])
Lib.wrap_func("sdp_pswf_generate", restype=None,
              argtypes=[_P, Mem.handle_type(), ctypes.c_int, ctypes.c_int],
              check_errcode=True)
