"""Status-code checking for wrapped C functions.

Same codes and "Error N: <meaning>" messages as the reference
(src/ska_sdp_func/utility/error_checking.py:11-46), which tests match on.
"""

import ctypes

ERROR_CODE_ARGTYPE = ctypes.POINTER(ctypes.c_int)

ERROR_CODE_MEANING = {
    0: "No error",
    1: "Generic runtime error",
    2: "Invalid function argument",
    3: "Unsupported data type(s)",
    4: "Memory allocation failure",
    5: "Memory copy failure",
    6: "Memory location mismatch",
}


class CError(Exception):
    """Raised when a wrapped C function returns a non-zero status."""


def error_checking(lib_func):
    """Wrap lib_func so that its trailing sdp_Error* status is checked."""

    def checked(*args):
        status = ctypes.c_int(0)
        result = lib_func(*args, ctypes.byref(status))
        if status.value:
            meaning = ERROR_CODE_MEANING.get(status.value, "Unknown error")
            raise CError(f"Error {status.value}: {meaning}")
        return result

    checked.__name__ = getattr(lib_func, "__name__", "wrapped")
    return checked
