"""Locate libska_sdp_func and expose its C functions lazily.

Behaviour follows the reference loader (src/ska_sdp_func/utility/lib.py):
the library is found by globbing "libska_sdp_func*" in $SKA_SDP_FUNC_LIB_DIR,
the current directory, the package root and /usr/local/lib; functions are
declared with Lib.wrap_func(name, restype=..., argtypes=[...],
check_errcode=...) and bound on first access as Lib.<name>.

MI355X note: if PyTorch is importable it is imported BEFORE the library is
loaded, so that the process has exactly one HIP runtime (the library's
libamdhip64.so.7 dependency then resolves to the copy torch already loaded).
"""

import ctypes
import glob
import os
import threading

from .error_checking import ERROR_CODE_ARGTYPE, error_checking


class _LibMeta(type):
    def __getattr__(cls, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return cls._bind(name)


class Lib(metaclass=_LibMeta):
    """Handle to the compiled library; wrapped C functions are attributes."""

    name = "libska_sdp_func"
    env_name = "SKA_SDP_FUNC_LIB_DIR"
    package_root = os.path.abspath(
        os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
    )
    search_dirs = [".", package_root, "/usr/local/lib"]
    lib = None
    _lock = threading.Lock()
    _specs = {}

    @staticmethod
    def find_lib(dirs):
        """Return the first libska_sdp_func* found in dirs (or "")."""
        env_dir = os.environ.get(Lib.env_name)
        if env_dir and env_dir not in dirs:
            dirs.insert(0, env_dir)
        for d in dirs:
            hits = sorted(glob.glob(os.path.join(d, Lib.name) + "*"))
            hits = [h for h in hits if not h.endswith(".tmp")]
            if hits:
                return os.path.abspath(hits[0])
        return ""

    @staticmethod
    def handle():
        """Load (once) and return the ctypes handle of the library."""
        if Lib.lib is None:
            with Lib._lock:
                if Lib.lib is None:
                    try:  # one HIP runtime per process: torch's, if present
                        import torch  # noqa: F401
                    except ImportError:
                        pass
                    path = Lib.find_lib(Lib.search_dirs)
                    try:
                        Lib.lib = ctypes.CDLL(path) if path else None
                    except OSError:
                        Lib.lib = None
                    if Lib.lib is None:
                        raise RuntimeError(
                            f"Cannot find {Lib.name} in {Lib.search_dirs}. "
                            f"Try setting the environment variable "
                            f"{Lib.env_name}"
                        )
        return Lib.lib

    @staticmethod
    def wrap_func(func_name, *, restype, argtypes, check_errcode=False):
        """Declare the C signature of func_name (bound on first use)."""
        Lib._specs[func_name] = (restype, list(argtypes), check_errcode)

    @staticmethod
    def _bind(func_name):
        try:
            restype, argtypes, check = Lib._specs[func_name]
        except KeyError as err:
            raise KeyError(
                f"The wrapping details for {func_name!r} have not been defined"
            ) from err
        try:
            func = getattr(Lib.handle(), func_name)
        except AttributeError as err:
            raise AttributeError(
                f"The C library does not expose a function named {func_name!r}"
            ) from err
        func.restype = restype
        func.argtypes = argtypes + ([ERROR_CODE_ARGTYPE] if check else [])
        bound = error_checking(func) if check else func
        setattr(Lib, func_name, bound)
        return bound
