"""Deconvolution (mirror of src/ska_sdp_func/clean)."""

from .hogbom_clean import hogbom_clean

__all__ = ["hogbom_clean"]
