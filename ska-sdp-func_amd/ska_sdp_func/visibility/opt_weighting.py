"""Tiled Briggs weighting (MI355X HIP implementation).

Mirrors src/ska_sdp_func/visibility/opt_weighting.py of ska-sdp-func
1.2.2: same function names and arguments. All arrays on the GPU (torch or
cupy); the sorted arrays and tile_offsets are those written by
bucket_sort / tiled_indexing (visibility.tiled_functions). Semantics and
the reference defects not carried over: include/ska-sdp-func/visibility/
sdp_opt_weighting.h.
"""
import ctypes

from ..utility import Lib, Mem

Lib.wrap_func(
    "sdp_optimized_weighting",
    restype=None,
    argtypes=[Mem.handle_type()] * 4 + [
        ctypes.c_double, ctypes.c_int, ctypes.c_int64]
    + [Mem.handle_type()] * 7,
    check_errcode=True,
)

Lib.wrap_func(
    "sdp_optimised_indexed_weighting",
    restype=None,
    argtypes=[Mem.handle_type()] * 3 + [
        ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_int64,
        ctypes.POINTER(ctypes.c_int)] + [Mem.handle_type()] * 7,
    check_errcode=True,
)


def optimized_weighting(uvw, freqs, vis, weights, robust_param, grid_size,
                        support, sorted_uu, sorted_vv, sorted_weight,
                        sorted_tile, tile_offsets, num_points_in_tiles,
                        output_weights):
    """Briggs weights per 32 x 16 tile of bucket-sorted visibilities,
    written in sorted order into output_weights ([num sorted entries])."""
    Lib.sdp_optimized_weighting(
        Mem(uvw), Mem(freqs), Mem(vis), Mem(weights), robust_param,
        grid_size, support, Mem(sorted_uu), Mem(sorted_vv),
        Mem(sorted_weight), Mem(sorted_tile), Mem(tile_offsets),
        Mem(num_points_in_tiles), Mem(output_weights),
    )


def optimised_indexed_weighting(uvw, vis, weights, robust_param, grid_size,
                                cell_size_rad, support, num_visibilities,
                                sorted_tile, sorted_uu, sorted_vv,
                                sorted_vis_index, tile_offsets,
                                num_points_in_tiles, output_weights):
    """Briggs weights per tile through the sorted visibility indices,
    written into output_weights (shape of weights); num_visibilities is
    the ctypes.c_int filled by count_and_prefix_sum."""
    Lib.sdp_optimised_indexed_weighting(
        Mem(uvw), Mem(vis), Mem(weights), robust_param, grid_size,
        cell_size_rad, support, ctypes.byref(num_visibilities),
        Mem(sorted_tile), Mem(sorted_uu), Mem(sorted_vv),
        Mem(sorted_vis_index), Mem(tile_offsets), Mem(num_points_in_tiles),
        Mem(output_weights),
    )
