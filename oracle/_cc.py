"""TEST INFRASTRUCTURE ONLY -- compiles the C oracles (oracle/*.c) into
shared libraries for ctypes.

Default: gcc with the flags each oracle asks for, into oracle/_build.
With SDP_SANITIZE=1 (scripts/sanitize.sh, the SURVEY 5 sanitizer run): the
same sources built by the ROCm clang with AddressSanitizer and
UndefinedBehaviorSanitizer into oracle/_build_san, so that one process can
preload clang's ASan runtime for both the oracles and the sanitized
library (ska-sdp-func_amd/san).
"""
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LLVM = "/opt/rocm/lib/llvm"


def sanitize():
    return os.environ.get("SDP_SANITIZE") == "1"


def shared(src_name, lib_name, flags, force=False):
    """Build oracle/<src_name> into <build dir>/<lib_name> if out of date;
    return the library path."""
    san = sanitize()
    build = os.path.join(_HERE, "_build_san" if san else "_build")
    src = os.path.join(_HERE, src_name)
    lib = os.path.join(build, lib_name)
    if (not force and os.path.exists(lib)
            and os.path.getmtime(lib) >= os.path.getmtime(src)):
        return lib
    os.makedirs(build, exist_ok=True)
    tmp = lib + f".tmp{os.getpid()}"
    if san:
        cmd = [os.path.join(_LLVM, "bin", "clang"), "-g",
               "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
               "-shared-libsan", *flags, "-fPIC", "-shared", src, "-o", tmp,
               "-lm", f"-Wl,-rpath,{_LLVM}/lib"]
    else:
        cmd = ["gcc", *flags, "-fPIC", "-shared", src, "-o", tmp, "-lm"]
    subprocess.check_call(cmd)
    os.replace(tmp, lib)
    return lib
