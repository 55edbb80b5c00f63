"""Tiling and bucket sort of visibilities (MI355X HIP implementation).

Mirrors src/ska_sdp_func/visibility/tiled_functions.py of ska-sdp-func
1.2.2: same function names and arguments. All arrays on the GPU (torch or
cupy); num_visibilities is a ctypes.c_int filled by count_and_prefix_sum.
Semantics: the reference GPU kernels' tile arithmetic, entries within a
tile in visibility order (see include/ska-sdp-func/visibility/
sdp_tiled_functions.h).
"""
import ctypes

from ..utility import Lib, Mem

Lib.wrap_func(
    "sdp_count_and_prefix_sum",
    restype=None,
    argtypes=[Mem.handle_type()] * 3 + [
        ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_double,
        ctypes.c_int64, ctypes.POINTER(ctypes.c_int)] + [Mem.handle_type()] * 3,
    check_errcode=True,
)

Lib.wrap_func(
    "sdp_bucket_sort",
    restype=None,
    argtypes=[Mem.handle_type()] * 4 + [
        ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_double,
        ctypes.c_int64] + [Mem.handle_type()] * 6,
    check_errcode=True,
)

Lib.wrap_func(
    "sdp_tiled_indexing",
    restype=None,
    argtypes=[Mem.handle_type()] * 2 + [
        ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_double,
        ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64]
    + [Mem.handle_type()] * 5,
    check_errcode=True,
)


def count_and_prefix_sum(uvw, freqs, vis, grid_size, tile_size_u,
                         tile_size_v, cell_size_rad, support,
                         num_visibilities, tile_offsets, num_points_in_tiles,
                         num_skipped):
    """Entries per tile (num_points_in_tiles), their exclusive prefix sum
    plus total (tile_offsets, num_tiles + 1), visibilities off the grid
    (num_skipped) and the total into num_visibilities (ctypes.c_int)."""
    Lib.sdp_count_and_prefix_sum(
        Mem(uvw), Mem(freqs), Mem(vis), grid_size, tile_size_u, tile_size_v,
        cell_size_rad, support, ctypes.byref(num_visibilities),
        Mem(tile_offsets), Mem(num_points_in_tiles), Mem(num_skipped),
    )


def bucket_sort(uvw, freqs, vis, weights, grid_size, tile_size_u,
                tile_size_v, cell_size_rad, support, sorted_uu, sorted_vv,
                sorted_weight, sorted_tile, sorted_vis, tile_offsets):
    """Visibilities listed per tile (duplicated where they overlap several
    tiles) from tile_offsets, which advance to each tile's end."""
    Lib.sdp_bucket_sort(
        Mem(uvw), Mem(freqs), Mem(vis), Mem(weights), grid_size,
        tile_size_u, tile_size_v, cell_size_rad, support, Mem(sorted_uu),
        Mem(sorted_vv), Mem(sorted_weight), Mem(sorted_tile),
        Mem(sorted_vis), Mem(tile_offsets),
    )


def tiled_indexing(uvw, freqs, grid_size, tile_size_u, tile_size_v,
                   cell_size_rad, support, num_channels, num_baselines,
                   num_times, sorted_tile, sorted_uu, sorted_vv,
                   sorted_vis_index, tile_offsets):
    """As bucket_sort, listing visibility indices instead of values."""
    Lib.sdp_tiled_indexing(
        Mem(uvw), Mem(freqs), grid_size, tile_size_u, tile_size_v,
        cell_size_rad, support, num_channels, num_baselines, num_times,
        Mem(sorted_tile), Mem(sorted_uu), Mem(sorted_vv),
        Mem(sorted_vis_index), Mem(tile_offsets),
    )
