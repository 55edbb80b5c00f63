"""Utility classes (reference: src/ska_sdp_func/utility/__init__.py)."""

from .error_checking import CError
from .lib import Lib
from .mem import Mem
from .struct_wrapper import StructWrapper

__all__ = ["CError", "Lib", "Mem", "StructWrapper"]
