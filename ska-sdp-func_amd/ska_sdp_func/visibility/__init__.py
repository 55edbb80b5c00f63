"""Visibility-domain functions (mirror of src/ska_sdp_func/visibility)."""

from .flagger import flagger_dynamic_threshold
from .weighting import briggs_weights, get_uv_range, uniform_weights

__all__ = [
    "flagger_dynamic_threshold",
    "briggs_weights",
    "get_uv_range",
    "uniform_weights",
]
