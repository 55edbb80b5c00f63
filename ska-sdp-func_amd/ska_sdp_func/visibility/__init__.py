"""Visibility-domain functions (mirror of src/ska_sdp_func/visibility)."""

from .dft import dft_point_v00, dft_point_v01
from .flagger import flagger_dynamic_threshold
from .opt_weighting import optimised_indexed_weighting, optimized_weighting
from .tiled_functions import (bucket_sort, count_and_prefix_sum,
                              tiled_indexing)
from .weighting import briggs_weights, get_uv_range, uniform_weights

__all__ = [
    "dft_point_v00",
    "dft_point_v01",
    "flagger_dynamic_threshold",
    "briggs_weights",
    "get_uv_range",
    "uniform_weights",
    "bucket_sort",
    "count_and_prefix_sum",
    "tiled_indexing",
    "optimized_weighting",
    "optimised_indexed_weighting",
]
