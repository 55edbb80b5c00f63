"""FFT functions (reference: src/ska_sdp_func/fourier_transforms/
__init__.py); the SwiFTly transforms are out of scope."""

from .fft import (Fft, fft_2d_inplace_permuted, fft_permuted_n2,
                  padded_fft_size)

__all__ = ["Fft", "padded_fft_size", "fft_2d_inplace_permuted",
           "fft_permuted_n2"]
from .pswf import Pswf, generate_pswf  # noqa: E402

__all__ += ["Pswf", "generate_pswf"]
