"""CPU tests of the drop-in boundary (no GPU needed).

* libska_sdp_func.so loads and exports every function include/*.h declares;
* the sdp_Mem C ABI behaves like the reference's (utility/sdp_mem.cpp);
* the Python wrapper raises the reference's error strings for the argument
  checks of sdp_gridder_check_buffers (sdp_gridder_uvw_es_fft.cpp:72-262),
  mirroring the reference's test_gridder_plan
  (tests/grid_data/test_gridder_uvw_es_fft.py:21-431);
* the kernel-parameter selection of the library equals the reference's
  (golden vectors from the reference's own code).
"""
import ctypes
import glob
import json
import os
import re
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(ROOT, "ska-sdp-func_amd", "libska_sdp_func.so")


def _declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "**", "*.h"),
                       recursive=True):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        text = re.sub(r"//[^\n]*", "", text)
        text = re.sub(r"#define[^\n]*(\\\n[^\n]*)*", "", text)
        # Header-only (SDP_INLINE) functions are not library exports.
        inline = set(re.findall(r"SDP_INLINE\s+\w+\s+(sdp_[a-z0-9_]+)\s*\(",
                                text))
        for m in re.finditer(r"\b(sdp_[a-z0-9_]+)\s*\(", text):
            if m.group(1) not in inline:
                names.add(m.group(1))
    return names


# Every header path of the reference (ska-sdp-func 1.2.2, src/ska-sdp-func/)
# that a C / C++ caller of the hot path and its SURVEY 8 rows includes.
REFERENCE_HEADER_PATHS = [
    "utility/sdp_mem.h", "utility/sdp_errors.h", "utility/sdp_logging.h",
    "math/sdp_math_macros.h",
    "fourier_transforms/sdp_fft.h", "fourier_transforms/sdp_fft_padded_size.h",
    "fourier_transforms/sdp_pswf.h",
    "grid_data/sdp_gridder_uvw_es_fft.h", "grid_data/sdp_gridder_wtower_uvw.h",
    "grid_data/sdp_grid_wstack_wtower.h", "grid_data/sdp_gridder_utils.h",
    "grid_data/sdp_gridder_clamp_channels.h",
    "grid_data/sdp_gridder_wtower_height.h",
    "grid_data/sdp_gridder_grid_correct.h",
    "grid_data/sdp_degrid_uvw_custom.h",
    "visibility/sdp_flagger.h", "visibility/sdp_weighting.h",
    "visibility/sdp_tiled_functions.h", "visibility/sdp_opt_weighting.h",
    "visibility/sdp_dft.h",
    "clean/sdp_hogbom_clean.h", "clean/sdp_ms_clean_cornwell.h",
]


def test_reference_header_paths_exist():
    missing = [h for h in REFERENCE_HEADER_PATHS if not os.path.exists(
        os.path.join(ROOT, "include", "ska-sdp-func", h))]
    assert not missing, f"reference header paths missing: {missing}"


@pytest.mark.parametrize("lang", ["c", "c++"])
def test_headers_compile_like_a_caller(tmp_path, lang):
    """Every header, included by its reference path, compiles for a C (C99)
    and a C++ (C++11) caller, all together in one translation unit."""
    hdrs = sorted(os.path.relpath(h, os.path.join(ROOT, "include"))
                  for h in glob.glob(os.path.join(ROOT, "include", "**",
                                                  "*.h"), recursive=True))
    src = tmp_path / ("all.c" if lang == "c" else "all.cpp")
    src.write_text("".join(f'#include "{h}"\n' for h in hdrs)
                   + "int main(void) { return 0; }\n")
    cc, std = ("gcc", "-std=c99") if lang == "c" else ("g++", "-std=c++11")
    r = subprocess.run([cc, std, "-Wall", "-Werror", "-fsyntax-only",
                        "-I", os.path.join(ROOT, "include"), str(src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_clamp_channels_inline_matches_oracle(tmp_path):
    """The header-only sdp_gridder_clamp_channels_inline, compiled as C,
    against the oracle's restatement of the reference inline
    (sdp_gridder_clamp_channels.h:116-172) on random and edge cases."""
    from oracle import wtower_oracle as wo

    rng = np.random.default_rng(3)
    cases = []
    for _ in range(3000):
        u = float(rng.choice([0.0, 1e-9, -1e-9]) if rng.random() < 0.1
                  else rng.normal(0, 3000))
        f0 = float(rng.uniform(1e8, 2e9))
        df = float(rng.choice([0.0, 1e3]) if rng.random() < 0.1
                   else rng.uniform(-5e6, 5e6))
        s0, e0 = int(rng.integers(0, 50)), int(rng.integers(0, 400))
        lo = float(rng.normal(0, 5000))
        hi = lo + float(rng.choice([0.0, rng.uniform(0, 8000)]))
        cases.append((u, f0, df, s0, e0, lo, hi))
    inp = tmp_path / "in.txt"
    inp.write_text("".join("%r %r %r %d %d %r %r\n" % c for c in cases))
    src = tmp_path / "clamp.c"
    src.write_text(
        '#include <stdio.h>\n#include <stdint.h>\n'
        '#include "ska-sdp-func/grid_data/sdp_gridder_clamp_channels.h"\n'
        'int main(int argc, char** argv) {\n'
        '  FILE* f = fopen(argv[1], "r"); double u, f0, df, lo, hi;\n'
        '  long long s, e;\n'
        '  while (fscanf(f, "%lf %lf %lf %lld %lld %lf %lf", &u, &f0, &df,'
        ' &s, &e, &lo, &hi) == 7) {\n'
        '    int64_t a = s, b = e;\n'
        '    sdp_gridder_clamp_channels_inline(u, f0, df, &a, &b, lo, hi);\n'
        '    printf("%lld %lld\\n", (long long)a, (long long)b); }\n'
        '  return 0; }\n')
    exe = tmp_path / "clamp"
    subprocess.run(["gcc", "-std=c99", "-O2", "-I",
                    os.path.join(ROOT, "include"), str(src), "-o", str(exe),
                    "-lm"], check=True)
    out = subprocess.check_output([str(exe), str(inp)], text=True).split()
    got = np.array(out, dtype=np.int64).reshape(-1, 2)
    nonempty = 0
    for (u, f0, df, s0, e0, lo, hi), (a, b) in zip(cases, got):
        ref = wo.clamp_channels(u, f0, df, s0, e0, lo, hi)
        assert (a, b) == tuple(int(x) for x in ref), (u, f0, df, s0, e0, lo,
                                                     hi)
        nonempty += b > a
    assert nonempty > 150


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build() has not produced libska_sdp_func.so"
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB],
                                  text=True)
    exported = {line.split()[-1] for line in out.splitlines() if line}
    declared = _declared_functions()
    assert len(declared) > 50
    missing = sorted(declared - exported)
    assert not missing, f"declared but not exported: {missing}"


def test_library_loads_without_gpu():
    lib = ctypes.CDLL(LIB)
    assert hasattr(lib, "sdp_grid_uvw_es_fft")


def test_params_from_epsilon_matches_reference_golden():
    lib = ctypes.CDLL(LIB)
    f = lib.sdp_gridder_uvw_es_fft_params_from_epsilon
    f.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_int,
                  ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                  ctypes.POINTER(ctypes.c_double)]
    with open(os.path.join(HERE, "golden", "es_params.json")) as fh:
        gold = json.load(fh)["params"]
    for p in gold:
        g, w, b = ctypes.c_int(), ctypes.c_int(), ctypes.c_double()
        f(p["eps"], p["N"], p["double"], g, w, b)
        assert (g.value, w.value, b.value) == (
            p["grid_size"], p["support"], p["beta"]), p


def test_mem_wrapper_semantics():
    from ska_sdp_func.utility import Lib, Mem

    lib = Lib.handle()
    lib.sdp_mem_shape_dim.restype = ctypes.c_int64
    lib.sdp_mem_shape_dim.argtypes = [Mem.handle_type(), ctypes.c_int32]
    lib.sdp_mem_stride_bytes_dim.restype = ctypes.c_int64
    lib.sdp_mem_stride_bytes_dim.argtypes = [Mem.handle_type(),
                                             ctypes.c_int32]
    lib.sdp_mem_is_c_contiguous.argtypes = [Mem.handle_type()]
    lib.sdp_mem_is_read_only.argtypes = [Mem.handle_type()]
    lib.sdp_mem_type.argtypes = [Mem.handle_type()]
    lib.sdp_mem_location.argtypes = [Mem.handle_type()]
    a = np.zeros((5, 7), np.complex64)
    m = Mem(a)
    assert lib.sdp_mem_shape_dim(m, 0) == 5
    assert lib.sdp_mem_shape_dim(m, 1) == 7
    assert lib.sdp_mem_stride_bytes_dim(m, 0) == 56
    assert lib.sdp_mem_is_c_contiguous(m) == 1
    assert lib.sdp_mem_type(m) == 36
    assert lib.sdp_mem_location(m) == 0
    t = Mem(a[:, ::2])
    assert lib.sdp_mem_is_c_contiguous(t) == 0
    ro = np.zeros(3, np.float32)
    ro.flags.writeable = False
    assert lib.sdp_mem_is_read_only(Mem(ro)) == 1
    with pytest.raises(TypeError):
        Mem(np.zeros(3, np.int16))
    Mem()   # empty wrapper, as the reference allows


def _case(dtype=np.float64, num_vis=100, num_chan=10, n=64):
    cdt = np.complex128 if dtype == np.float64 else np.complex64
    uvw = np.zeros((num_vis, 3), dtype)
    freq = (1e9 + np.arange(num_chan) * 1e8).astype(dtype)
    vis = np.zeros((num_vis, num_chan), cdt)
    wt = np.ones((num_vis, num_chan), dtype)
    dirty = np.zeros((n, n), dtype)
    return [uvw, freq, vis, wt, dirty]


def _plan(args, px=1e-5, py=1e-5):
    from ska_sdp_func.grid_data import GridderUvwEsFft

    return GridderUvwEsFft(*args, px, py, 1e-5, False)


@pytest.mark.parametrize("idx,bad,pattern", [
    (0, lambda a: a.astype(np.complex128), "Unsupported data type"),
    (1, lambda a: a.astype(np.complex128), "Unsupported data type"),
    (2, lambda a: a.real.copy(), "Unsupported data type"),
    (3, lambda a: a.astype(np.complex128), "Unsupported data type"),
    (4, lambda a: a.astype(np.complex128), "Unsupported data type"),
    (0, lambda a: np.ascontiguousarray(a[:, 0:2]), "Invalid function argument"),
    (0, lambda a: a[:-1], "Invalid function argument"),
    (1, lambda a: a[:-1], "Invalid function argument"),
    (3, lambda a: np.ascontiguousarray(a[:, 0:-2]),
     "Invalid function argument"),
    (4, lambda a: np.ascontiguousarray(a[:, 0:-1]),
     "Invalid function argument"),
    (0, lambda a: a.astype(np.float32), "Unsupported data type"),
    (1, lambda a: a.astype(np.float32), "Unsupported data type"),
    (2, lambda a: a.astype(np.complex64), "Unsupported data type"),
    (3, lambda a: a.astype(np.float32), "Unsupported data type"),
    (4, lambda a: a.astype(np.float32), "Unsupported data type"),
    (2, lambda a: a[:, ::2], "Invalid function argument"),
])
def test_create_plan_argument_checks(idx, bad, pattern):
    """Same error codes as the reference test_gridder_plan cases."""
    from ska_sdp_func.utility import CError

    args = _case()
    args[idx] = bad(args[idx])
    with pytest.raises(CError, match=pattern):
        _plan(args)


def test_pixel_sizes_must_match():
    from ska_sdp_func.utility import CError

    with pytest.raises(CError, match="Invalid function argument"):
        _plan(_case(), 1e-5, 2e-5)


def test_read_only_dirty_image_rejected():
    from ska_sdp_func.utility import CError

    args = _case()
    args[4].flags.writeable = False
    with pytest.raises(CError, match="Invalid function argument"):
        _plan(args)


def test_host_memory_has_no_cpu_fallback():
    """Host arrays end in 'Memory location mismatch' (at plan creation when
    no GPU is present, at the call otherwise) -- never a CPU computation."""
    from ska_sdp_func.utility import CError

    args = _case()
    with pytest.raises(CError, match="Memory location mismatch"):
        plan = _plan(args)
        plan.grid_uvw_es_fft(*args)


def test_get_w_range_numpy():
    """gridder_uvw_es_fft.py:90-106 semantics (reference test :315-372)."""
    from ska_sdp_func.grid_data import GridderUvwEsFft

    rng = np.random.default_rng(0)
    uvw = rng.uniform(-1000, 1000, (50, 3))
    freq = np.array([1e9, 1.5e9])
    lo, hi = GridderUvwEsFft.get_w_range(uvw, freq)
    assert lo == np.amin(np.abs(uvw[:, 2])) * 1e9 / 299792458.0
    assert hi == np.amax(np.abs(uvw[:, 2])) * 1.5e9 / 299792458.0
    assert GridderUvwEsFft.get_w_range([1, 2], freq) == (-1, -1)


# Flagger argument checks (sdp_flagger.cpp:10-57): all raised before any
# device work, so they run without a GPU.
def _flag_call(vis, flags, **over):
    from ska_sdp_func.visibility import flagger_dynamic_threshold

    kw = dict(alpha=0.5, threshold_magnitudes=3.5, threshold_variations=3.5,
              threshold_broadband=3.5, sampling_step=1, window=0,
              window_median_history=20)
    kw.update(over)
    flagger_dynamic_threshold(vis, flags, **kw)


def test_flagger_argument_errors():
    from ska_sdp_func.utility import CError

    vis = np.ones((4, 2, 8, 1), np.complex64)
    flags = np.zeros((4, 2, 8, 1), np.int32)
    with pytest.raises(CError, match="Error 1"):        # not 4-D
        _flag_call(vis[:, :, :, 0], flags[:, :, :, 0])
    with pytest.raises(CError, match="Error 1"):        # not contiguous
        _flag_call(vis[:, :, ::2], flags[:, :, ::2])
    with pytest.raises(CError, match="Error 3"):        # real vis
        _flag_call(np.ones((4, 2, 8, 1), np.float32), flags)
    with pytest.raises(CError, match="Error 3"):        # float flags
        _flag_call(vis, np.zeros((4, 2, 8, 1), np.float32))
    with pytest.raises(CError, match="Error 2"):        # shape mismatch
        _flag_call(vis, np.zeros((4, 2, 7, 1), np.int32))
    with pytest.raises(CError, match="Error 2"):        # sampling_step 0
        _flag_call(vis, flags, sampling_step=0)
    ro = flags.copy()
    ro.setflags(write=False)
    with pytest.raises(CError, match="Error 1"):        # read-only flags
        _flag_call(vis, ro)
