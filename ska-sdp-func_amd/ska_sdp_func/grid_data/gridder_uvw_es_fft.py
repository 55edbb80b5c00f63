"""ES-kernel + FFT (de)gridder, MI355X build.

Same class, methods and arguments as the reference
src/ska_sdp_func/grid_data/gridder_uvw_es_fft.py:16-200, bound to this
repository's libska_sdp_func (HIP / rocFFT). Device arrays may be torch
tensors on a ROCm device (or cupy arrays); host arrays are rejected by the
library with "Error 6: Memory location mismatch", as in the reference.
"""

import ctypes

import numpy as np

from ..utility import Lib, Mem, StructWrapper

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None

try:
    import cupy
except ImportError:
    cupy = None


class GridderUvwEsFft(StructWrapper):
    """Plan for (de)gridding with the exponential-of-semicircle kernel."""

    def __init__(
        self,
        uvw,
        freq_hz,
        vis,
        weight,
        dirty_image,
        pixel_size_x_rad,
        pixel_size_y_rad,
        epsilon: float,
        do_w_stacking: bool,
    ):
        """Create a plan; see the reference docstring for the arguments.

        uvw [num_rows, 3], freq_hz [num_chan], vis [num_rows, num_chan]
        complex, weight [num_rows, num_chan], dirty_image [N, N] (square);
        one precision for all; the precision of vis sets the precision of
        the computation. epsilon: requested accuracy (>= 1e-5 for single
        precision). do_w_stacking: full w-stacking if True, else w = 0.
        """
        if do_w_stacking:
            min_abs_w, max_abs_w = GridderUvwEsFft.get_w_range(uvw, freq_hz)
        else:
            min_abs_w = 0
            max_abs_w = 0
        create_args = (
            Mem(uvw),
            Mem(freq_hz),
            Mem(vis),
            Mem(weight),
            Mem(dirty_image),
            pixel_size_x_rad,
            pixel_size_y_rad,
            epsilon,
            float(min_abs_w),
            float(max_abs_w),
            do_w_stacking,
        )
        super().__init__(
            Lib.sdp_gridder_uvw_es_fft_create_plan,
            create_args,
            Lib.sdp_gridder_uvw_es_fft_free_plan,
        )

    @staticmethod
    def get_w_range(uvw, freq_hz):
        """Min / max |w| in wavelengths (gridder_uvw_es_fft.py:90-106)."""
        if isinstance(uvw, np.ndarray):
            min_abs_w = np.amin(np.abs(uvw[:, 2]))
            max_abs_w = np.amax(np.abs(uvw[:, 2]))
        elif torch is not None and isinstance(uvw, torch.Tensor):
            min_abs_w = torch.amin(torch.abs(uvw[:, 2])).item()
            max_abs_w = torch.amax(torch.abs(uvw[:, 2])).item()
        elif cupy and isinstance(uvw, cupy.ndarray):
            min_abs_w = cupy.amin(cupy.abs(uvw[:, 2]))
            max_abs_w = cupy.amax(cupy.abs(uvw[:, 2]))
        else:
            print(f"Unsupported uvw type of {type(uvw)}.")
            return -1, -1
        f_first = freq_hz[0]
        f_last = freq_hz[-1]
        if torch is not None and isinstance(freq_hz, torch.Tensor):
            f_first, f_last = f_first.item(), f_last.item()
        min_abs_w *= f_first / 299792458.0
        max_abs_w *= f_last / 299792458.0
        return min_abs_w, max_abs_w

    def grid_uvw_es_fft(self, uvw, freq_hz, vis, weight, dirty_image):
        """Grid visibilities into (accumulate onto) dirty_image."""
        Lib.sdp_grid_uvw_es_fft(
            self, Mem(uvw), Mem(freq_hz), Mem(vis), Mem(weight),
            Mem(dirty_image),
        )

    def ifft_grid_uvw_es(self, uvw, freq_hz, vis, weight, dirty_image):
        """Degrid dirty_image into (accumulate onto) vis.

        dirty_image is modified in place (grid correction), as in the
        reference.
        """
        Lib.sdp_ifft_degrid_uvw_es(
            self, Mem(uvw), Mem(freq_hz), Mem(vis), Mem(weight),
            Mem(dirty_image),
        )

    # ---- MI355X extensions ------------------------------------------------

    @property
    def grid_size(self):
        """Side of the (oversampled) uv grid."""
        return Lib.sdp_gridder_uvw_es_fft_grid_size(self)

    @property
    def support(self):
        """Kernel support W (cells)."""
        return Lib.sdp_gridder_uvw_es_fft_support(self)

    @property
    def num_w_planes(self):
        """Number of w-planes (1 without w-stacking)."""
        return Lib.sdp_gridder_uvw_es_fft_num_w_planes(self)

    @property
    def beta(self):
        """Full ES kernel beta."""
        return Lib.sdp_gridder_uvw_es_fft_beta(self)

    @property
    def fused_fft(self):
        """True if the plan uses the pruned, fused FFT passes (f32,
        power-of-two grid); False for rocFFT + separate screen kernels."""
        return bool(Lib.sdp_gridder_uvw_es_fft_fused_fft(self))

    def set_max_batch(self, max_vis):
        """Cap the visibilities bucketed together (0: the default cap);
        larger calls run in row batches (MI355X extension)."""
        Lib.sdp_gridder_uvw_es_fft_set_max_batch(self, int(max_vis))

    @property
    def batch_vis(self):
        """Visibilities per bucketing batch (MI355X extension)."""
        return int(Lib.sdp_gridder_uvw_es_fft_batch_vis(self))

    def set_stream(self, hip_stream_handle):
        """Launch on the given hipStream_t (int handle; 0 = null stream)."""
        Lib.sdp_gridder_uvw_es_fft_set_stream(
            self, ctypes.c_void_p(hip_stream_handle))

    def enable_timing(self, enable=True):
        """Record per-phase HIP-event timings of each call."""
        Lib.sdp_gridder_uvw_es_fft_enable_timing(self, int(enable))

    def get_timing(self):
        """Per-phase device ms of the last call (dict) or None."""
        out = (ctypes.c_double * 5)()
        n = Lib.sdp_gridder_uvw_es_fft_get_timing(self, out, 5)
        if n == 0:
            return None
        keys = ("bucket", "tile_kernel", "fft", "image", "total")
        return dict(zip(keys, list(out)[:n]))

    def grid_scatter(self, uvw, freq_hz, vis, weight, grid):
        """2-D only: scatter this process's rows into grid [G, G] complex."""
        Lib.sdp_grid_uvw_es_fft_scatter(
            self, Mem(uvw), Mem(freq_hz), Mem(vis), Mem(weight), Mem(grid))

    def grid_finish(self, grid, dirty_image):
        """2-D only: inverse FFT (in place) + screen + correction."""
        Lib.sdp_grid_uvw_es_fft_finish(self, Mem(grid), Mem(dirty_image))

    def row_spectra(self):
        """(rows, col0, ncols) of the grid block the column passes read
        after grid_rows, or None if the plan has no fused f32 FFT (f64 or
        non-power-of-two grids, 3-D). MI355X extension."""
        r, c, n = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        if not Lib.sdp_gridder_uvw_es_fft_row_spectra(
                self, ctypes.byref(r), ctypes.byref(c), ctypes.byref(n)):
            return None
        return r.value, c.value, n.value

    def grid_rows(self, grid):
        """First inverse-FFT pass (row FFTs) of a scattered grid, in place.
        Linear: row spectra of several grids may be summed before
        grid_finish_rows. MI355X extension."""
        Lib.sdp_grid_uvw_es_fft_rows(self, Mem(grid))

    def grid_finish_rows(self, grid, dirty_image):
        """Column passes + screen + correction of a grid after grid_rows:
        grid_scatter + grid_rows + grid_finish_rows == grid_scatter +
        grid_finish. MI355X extension."""
        Lib.sdp_grid_uvw_es_fft_finish_rows(self, Mem(grid),
                                            Mem(dirty_image))


_H = GridderUvwEsFft.handle_type()
_M = Mem.handle_type()

Lib.wrap_func(
    "sdp_gridder_uvw_es_fft_create_plan",
    restype=_H,
    argtypes=[_M, _M, _M, _M, _M, ctypes.c_double, ctypes.c_double,
              ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int],
    check_errcode=True,
)
Lib.wrap_func("sdp_gridder_uvw_es_fft_free_plan", restype=None, argtypes=[_H])
Lib.wrap_func("sdp_grid_uvw_es_fft", restype=None,
              argtypes=[_H, _M, _M, _M, _M, _M], check_errcode=True)
Lib.wrap_func("sdp_ifft_degrid_uvw_es", restype=None,
              argtypes=[_H, _M, _M, _M, _M, _M], check_errcode=True)
for _name in ("grid_size", "support", "num_w_planes"):
    Lib.wrap_func(f"sdp_gridder_uvw_es_fft_{_name}", restype=ctypes.c_int,
                  argtypes=[_H])
Lib.wrap_func("sdp_gridder_uvw_es_fft_beta", restype=ctypes.c_double,
              argtypes=[_H])
Lib.wrap_func("sdp_gridder_uvw_es_fft_fused_fft", restype=ctypes.c_int,
              argtypes=[_H])
Lib.wrap_func("sdp_gridder_uvw_es_fft_set_max_batch", restype=None,
              argtypes=[_H, ctypes.c_int64])
Lib.wrap_func("sdp_gridder_uvw_es_fft_batch_vis", restype=ctypes.c_int64,
              argtypes=[_H])
Lib.wrap_func("sdp_gridder_uvw_es_fft_set_stream", restype=None,
              argtypes=[_H, ctypes.c_void_p])
Lib.wrap_func("sdp_gridder_uvw_es_fft_enable_timing", restype=None,
              argtypes=[_H, ctypes.c_int])
Lib.wrap_func("sdp_gridder_uvw_es_fft_get_timing", restype=ctypes.c_int,
              argtypes=[_H, ctypes.POINTER(ctypes.c_double), ctypes.c_int])
Lib.wrap_func("sdp_grid_uvw_es_fft_scatter", restype=None,
              argtypes=[_H, _M, _M, _M, _M, _M], check_errcode=True)
Lib.wrap_func("sdp_grid_uvw_es_fft_finish", restype=None,
              argtypes=[_H, _M, _M], check_errcode=True)
Lib.wrap_func("sdp_gridder_uvw_es_fft_row_spectra", restype=ctypes.c_int,
              argtypes=[_H, ctypes.POINTER(ctypes.c_int64),
                        ctypes.POINTER(ctypes.c_int64),
                        ctypes.POINTER(ctypes.c_int64)])
Lib.wrap_func("sdp_grid_uvw_es_fft_rows", restype=None, argtypes=[_H, _M],
              check_errcode=True)
Lib.wrap_func("sdp_grid_uvw_es_fft_finish_rows", restype=None,
              argtypes=[_H, _M, _M], check_errcode=True)
