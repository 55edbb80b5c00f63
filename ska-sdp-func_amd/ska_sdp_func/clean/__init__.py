"""Deconvolution (mirror of src/ska_sdp_func/clean)."""

from .hogbom_clean import hogbom_clean
from .ms_clean_cornwell import ms_clean_cornwell

__all__ = ["hogbom_clean", "ms_clean_cornwell"]
