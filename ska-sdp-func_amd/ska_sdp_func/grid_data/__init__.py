"""Gridding functions (reference: src/ska_sdp_func/grid_data/__init__.py)."""

from .gridder_uvw_es_fft import GridderUvwEsFft

__all__ = ["GridderUvwEsFft"]
