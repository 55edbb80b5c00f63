"""Lifetime management of C structs returned by the library.

Same contract as src/ska_sdp_func/utility/struct_wrapper.py: each subclass
gets its own ctypes handle type (so handles cannot be mixed up), creation
returning NULL raises RuntimeError, and the free function runs when the
Python object is garbage collected.
"""

import ctypes
import weakref


class StructWrapper:
    """Base class of objects wrapping a C struct handle."""

    _HANDLE_CLASS = None

    def __init_subclass__(cls):
        cls._HANDLE_CLASS = type(f"{cls.__name__}Handle",
                                 (ctypes.Structure,), {})

    def __init__(self, create_func, create_args, free_func):
        if not callable(free_func):
            raise ValueError("free_func must be callable")
        self._handle = None
        handle = create_func(*create_args)
        if not handle:
            raise RuntimeError(
                "Cannot initialise struct wrapper: creation function for "
                f"{type(self).__name__} handle returned a null pointer"
            )
        self._handle = handle
        weakref.finalize(self, free_func, handle)

    @property
    def _as_parameter_(self):
        return self._handle

    @classmethod
    def handle_type(cls):
        """ctypes type to use in argtypes for this wrapper."""
        return ctypes.POINTER(cls._HANDLE_CLASS)
