"""FFT plans on rocFFT, MI355X build.

Same class, methods and arguments as the reference
src/ska_sdp_func/fourier_transforms/fft.py:13-92; the transform runs on the
GPU (host arrays are staged through device memory).
"""

import ctypes

from ..utility import Lib, Mem, StructWrapper


class Fft(StructWrapper):
    """Complex-to-complex FFT plan (sdp_fft_create / sdp_fft_exec)."""

    def __init__(self, input_data, output_data, num_dims_fft, is_forward):
        """Plan for the given arrays. With one more array dimension than
        num_dims_fft, the first dimension is the batch. Unnormalised in
        both directions (inverse = +i exponent)."""
        create_args = (
            Mem(input_data),
            Mem(output_data),
            num_dims_fft,
            is_forward,
        )
        super().__init__(Lib.sdp_fft_create, create_args, Lib.sdp_fft_free)

    def exec(self, input_data, output_data):
        """Transform input_data into output_data (arrays matching the
        plan's)."""
        Lib.sdp_fft_exec(self, Mem(input_data), Mem(output_data))

    def exec_shift(self, data, norm=False):
        """phase, FFT in place, phase, and 1 / N if norm (sdp_fft.h:94)."""
        Lib.sdp_fft_exec_shift(self, Mem(data), int(bool(norm)))


def padded_fft_size(num: int, padding_factor: float):
    """The smallest even number >= ceil(num * padding_factor) whose half
    has no prime factor above 11."""
    return Lib.sdp_fft_padded_size(num, padding_factor)


def fft_norm(data):
    """data *= 1 / (dim0 * dim1) (sdp_fft_norm)."""
    Lib.sdp_fft_norm(Mem(data))


def fft_phase(data):
    """data *= (-1)^(i + j) (sdp_fft_phase)."""
    Lib.sdp_fft_phase(Mem(data))


def fft_2d_inplace_permuted(data, is_forward):
    """MI355X extension: the w-stack plane FFT in place on a square
    complex64 GPU array (side a power of two in [1024, 16384]); output row
    k is stored at row N1 * (k % N2) + k // N2, N2 = fft_permuted_n2(G)."""
    Lib.sdp_fft_2d_inplace_permuted(Mem(data), int(bool(is_forward)))


def fft_permuted_n2(grid_size):
    """N2 of sdp_fft_2d_inplace_permuted's row permutation (0: size not
    supported)."""
    return int(Lib.sdp_fft_permuted_n2(int(grid_size)))


Lib.wrap_func(
    "sdp_fft_create",
    restype=Fft.handle_type(),
    argtypes=[
        Mem.handle_type(),
        Mem.handle_type(),
        ctypes.c_int32,
        ctypes.c_int32,
    ],
    check_errcode=True,
)

Lib.wrap_func(
    "sdp_fft_free",
    restype=None,
    argtypes=[Fft.handle_type()],
)

Lib.wrap_func(
    "sdp_fft_exec",
    restype=None,
    argtypes=[
        Fft.handle_type(),
        Mem.handle_type(),
        Mem.handle_type(),
    ],
    check_errcode=True,
)

Lib.wrap_func(
    "sdp_fft_exec_shift",
    restype=None,
    argtypes=[Fft.handle_type(), Mem.handle_type(), ctypes.c_int],
    check_errcode=True,
)

Lib.wrap_func(
    "sdp_fft_norm",
    restype=None,
    argtypes=[Mem.handle_type()],
    check_errcode=True,
)

Lib.wrap_func(
    "sdp_fft_phase",
    restype=None,
    argtypes=[Mem.handle_type()],
    check_errcode=True,
)

Lib.wrap_func(
    "sdp_fft_padded_size",
    restype=ctypes.c_int,
    argtypes=[
        ctypes.c_int,
        ctypes.c_double,
    ],
)

Lib.wrap_func(
    "sdp_fft_2d_inplace_permuted",
    restype=None,
    argtypes=[Mem.handle_type(), ctypes.c_int],
    check_errcode=True,
)

Lib.wrap_func(
    "sdp_fft_permuted_n2",
    restype=ctypes.c_int,
    argtypes=[ctypes.c_int],
)
