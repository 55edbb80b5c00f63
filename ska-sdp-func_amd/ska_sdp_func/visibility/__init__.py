"""Visibility-domain functions (mirror of src/ska_sdp_func/visibility)."""

from .flagger import flagger_dynamic_threshold

__all__ = ["flagger_dynamic_threshold"]
