"""Mem: wraps an array as an sdp_Mem for the processing functions.

Accepts numpy arrays (host memory), torch tensors (ROCm device memory when
tensor.is_cuda, host otherwise) and cupy arrays if cupy is installed. Type
codes and byte strides are those of the reference
(src/ska_sdp_func/utility/mem.py:18-136, utility/sdp_mem.h:73-113).
"""

import ctypes

import numpy

from .lib import Lib
from .struct_wrapper import StructWrapper

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None

try:
    import cupy
except ImportError:
    cupy = None


class Mem(StructWrapper):
    """Non-owning sdp_Mem view of an array."""

    class MemType:
        """sdp_MemType codes."""

        SDP_MEM_VOID = 0
        SDP_MEM_CHAR = 1
        SDP_MEM_INT = 2
        SDP_MEM_FLOAT = 4
        SDP_MEM_DOUBLE = 8
        SDP_MEM_COMPLEX_FLOAT = 36
        SDP_MEM_COMPLEX_DOUBLE = 40

    class MemLocation:
        """sdp_MemLocation codes."""

        SDP_MEM_CPU = 0
        SDP_MEM_GPU = 1

    _NUMPY_TYPES = {
        numpy.dtype(numpy.int8): MemType.SDP_MEM_CHAR,
        numpy.dtype(numpy.int32): MemType.SDP_MEM_INT,
        numpy.dtype(numpy.float32): MemType.SDP_MEM_FLOAT,
        numpy.dtype(numpy.float64): MemType.SDP_MEM_DOUBLE,
        numpy.dtype(numpy.complex64): MemType.SDP_MEM_COMPLEX_FLOAT,
        numpy.dtype(numpy.complex128): MemType.SDP_MEM_COMPLEX_DOUBLE,
    }

    def __init__(self, *args):
        obj = args[0] if len(args) == 1 else None
        if obj is None:
            one = (ctypes.c_int64 * 1)(1)
            create = (ctypes.c_void_p(), self.MemType.SDP_MEM_VOID,
                      self.MemLocation.SDP_MEM_CPU, 0, one, one)
            super().__init__(Lib.sdp_mem_create_wrapper, create,
                             Lib.sdp_mem_free)
            return
        if isinstance(obj, numpy.ndarray):
            mem_type = self._type_of(obj.dtype, "numpy")
            ptr = obj.ctypes.data
            loc = self.MemLocation.SDP_MEM_CPU
            shape, strides = obj.shape, obj.strides
            read_only = not obj.flags.writeable
        elif torch is not None and isinstance(obj, torch.Tensor):
            mem_type = self._type_of(self._torch_dtype(obj.dtype), "torch")
            ptr = obj.data_ptr()
            if ptr == 0 and obj.numel() == 0:
                # torch reports NULL for empty views; pass the allocation's
                # address (never dereferenced), as numpy does for empty
                # arrays, so that the C side's type checks (which treat a
                # NULL array as untyped, sdp_mem.cpp:643-647) see the dtype.
                ptr = obj.untyped_storage().data_ptr()
            loc = (self.MemLocation.SDP_MEM_GPU if obj.is_cuda
                   else self.MemLocation.SDP_MEM_CPU)
            shape = tuple(obj.shape)
            strides = tuple(s * obj.element_size() for s in obj.stride())
            read_only = False
        elif cupy is not None and isinstance(obj, cupy.ndarray):
            mem_type = self._type_of(numpy.dtype(obj.dtype), "cupy")
            ptr = obj.data.ptr
            loc = self.MemLocation.SDP_MEM_GPU
            shape, strides = obj.shape, obj.strides
            read_only = False
        else:
            raise TypeError("Unsupported argument type")
        self._keep = obj  # keep the data alive while the wrapper exists
        ndim = len(shape)
        c_shape = (ctypes.c_int64 * max(ndim, 1))(*shape)
        c_strides = (ctypes.c_int64 * max(ndim, 1))(*strides)
        create = (ctypes.c_void_p(ptr), mem_type, loc, ndim, c_shape,
                  c_strides)
        super().__init__(Lib.sdp_mem_create_wrapper, create, Lib.sdp_mem_free)
        Lib.sdp_mem_set_read_only(self, int(read_only))

    @classmethod
    def _type_of(cls, dtype, kind):
        try:
            return cls._NUMPY_TYPES[numpy.dtype(dtype)]
        except (KeyError, TypeError) as err:
            raise TypeError(f"Unsupported type of {kind} array") from err

    @staticmethod
    def _torch_dtype(dtype):
        table = {
            torch.int8: numpy.int8, torch.int32: numpy.int32,
            torch.float32: numpy.float32, torch.float64: numpy.float64,
            torch.complex64: numpy.complex64,
            torch.complex128: numpy.complex128,
        }
        if dtype not in table:
            raise TypeError("Unsupported type of torch tensor")
        return table[dtype]


Lib.wrap_func(
    "sdp_mem_create_wrapper",
    restype=Mem.handle_type(),
    argtypes=[ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int32,
              ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)],
    check_errcode=True,
)
Lib.wrap_func("sdp_mem_set_read_only", restype=None,
              argtypes=[Mem.handle_type(), ctypes.c_int32])
Lib.wrap_func("sdp_mem_free", restype=None, argtypes=[Mem.handle_type()])
