"""Gridding functions (reference: src/ska_sdp_func/grid_data/__init__.py)."""

from .degrid_uvw_custom import degrid_uvw_custom
from .gridder_utils import (
    clamp_channels_single,
    clamp_channels_uv,
    determine_max_w_tower_height,
    determine_w_step,
    find_max_w_tower_height,
    make_kernel,
    make_pswf_kernel,
    make_w_pattern,
    rms_diff,
    subgrid_add,
    subgrid_cut_out,
    uvw_bounds_all,
)
from .grid_wstack_wtower import (
    wstack_wtower_degrid_all,
    wstack_wtower_degrid_planes,
    wstack_wtower_enable_timing,
    wstack_wtower_get_timing,
    wstack_wtower_grid_all,
    wstack_wtower_grid_planes,
)
from .gridder_uvw_es_fft import GridderUvwEsFft
from .gridder_wtower_uvw import GridderWtowerUVW

__all__ = [
    "GridderUvwEsFft",
    "GridderWtowerUVW",
    "clamp_channels_single",
    "degrid_uvw_custom",
    "clamp_channels_uv",
    "determine_max_w_tower_height",
    "determine_w_step",
    "find_max_w_tower_height",
    "make_kernel",
    "make_pswf_kernel",
    "make_w_pattern",
    "rms_diff",
    "subgrid_add",
    "subgrid_cut_out",
    "uvw_bounds_all",
    "wstack_wtower_degrid_all",
    "wstack_wtower_degrid_planes",
    "wstack_wtower_enable_timing",
    "wstack_wtower_get_timing",
    "wstack_wtower_grid_all",
    "wstack_wtower_grid_planes",
]
