"""Visibility weighting (csrc/visibility/sdp_weighting.hip) against the CPU
oracle (oracle/weighting_oracle.py, a restatement of sdp_weighting.cpp).

CPU tests pin the oracle: its vectorised form against its plain-loop form
in the reference's loop order, and a known answer derived by hand for the
reference test's prime_3x3 input (every visibility lands in cell (1, 1):
grid = 3 (10 + 31 + 21) = 186, uniform weights 1 / 186, Briggs at
robust = -2: R = 500^2 / 186, so out = w / 250001). GPU tests compare the
HIP functions with the oracle on host (staged) and device arrays:
float64 to 1e-12 relative (the grid sums are accumulated with atomics in a
different order), float32 to 1e-5 (f32 atomics reorder the grid sums).
"""
import numpy as np
import pytest

import weight_data as wd
from oracle import weighting_oracle as wo


def _run_oracle(case, G, robust, loops=False, dtype=np.float64):
    freqs, uvw, mx, inp = case
    inp = inp.astype(dtype)
    grid = np.zeros((G, G, inp.shape[3]), dtype)
    out = np.full(inp.shape, -7.0, dtype)
    f = wo.weighting_loops if loops else wo.weighting
    f(uvw, freqs, mx, grid, inp, out, robust)
    return grid, out


@pytest.mark.parametrize("robust", [None, -2.0, 0.0, 1.5])
@pytest.mark.parametrize("case,G", [("prime", 3), ("flat", 4),
                                    ("random", 16)])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_oracle_vectorised_matches_loops(case, G, robust, dtype):
    c = {"prime": wd.prime_case, "flat": wd.flat_case,
         "random": lambda: wd.random_case(T=4, B=10, C=3)}[case]()
    g1, o1 = _run_oracle(c, G, robust, dtype=dtype)
    g2, o2 = _run_oracle(c, G, robust, loops=True, dtype=dtype)
    assert np.array_equal(g1, g2)
    assert np.array_equal(o1, o2)


def test_oracle_known_answer():
    c = wd.prime_case()
    grid, out = _run_oracle(c, 3, None)
    assert grid[1, 1, 0] == 186.0 and np.count_nonzero(grid) == 1
    assert np.all(out == 1.0 / 186.0)
    grid, out = _run_oracle(c, 3, -2.0)
    np.testing.assert_allclose(out, c[3] / 250001.0, rtol=1e-14)


def test_library_exports_weighting():
    from ska_sdp_func.utility import Lib
    lib = Lib.handle()
    for name in ("sdp_weighting_uniform", "sdp_weighting_briggs"):
        assert hasattr(lib, name)


# -- GPU -------------------------------------------------------------------

def _gpu(case, G, robust, dtype, device=None):
    from ska_sdp_func.visibility import briggs_weights, uniform_weights
    freqs, uvw, mx, inp = case
    inp = inp.astype(dtype)
    grid = np.zeros((G, G, inp.shape[3]), dtype)
    out = np.full(inp.shape, -7.0, dtype)
    args = [uvw, freqs, mx]
    arrays = [grid, inp, out]
    if device is not None:
        import torch
        args[0] = torch.from_numpy(uvw).to(device)
        args[1] = torch.from_numpy(freqs).to(device)
        arrays = [torch.from_numpy(a).to(device) for a in arrays]
    if robust is None:
        uniform_weights(*args, *arrays)
    else:
        briggs_weights(*args[:3], robust, *arrays)
    if device is not None:
        import torch
        torch.cuda.synchronize()
        arrays = [a.cpu().numpy() for a in arrays]
    return arrays[0], arrays[2]


@pytest.mark.gpu
@pytest.mark.parametrize("robust", [None, -2.0, 0.5])
@pytest.mark.parametrize("dtype,rtol", [(np.float64, 1e-12),
                                        (np.float32, 1e-5)])
@pytest.mark.parametrize("on_device", [False, True])
def test_gpu_matches_oracle(device, robust, dtype, rtol, on_device):
    for case, G in ((wd.prime_case(), 3), (wd.flat_case(), 4),
                    (wd.random_case(), 64),
                    (wd.random_case(T=200, B=300, C=16, P=4, seed=9), 512)):
        g_ref, o_ref = _run_oracle(case, G, robust, dtype=dtype)
        g, o = _gpu(case, G, robust, dtype, device if on_device else None)
        np.testing.assert_allclose(g, g_ref, rtol=rtol, atol=0)
        np.testing.assert_allclose(o, o_ref, rtol=rtol, atol=0)


@pytest.mark.gpu
def test_gpu_argument_errors(device):
    from ska_sdp_func.utility import CError
    from ska_sdp_func.visibility import uniform_weights
    freqs, uvw, mx, inp = wd.prime_case()
    grid = np.zeros((3, 3, 1))
    out = np.zeros_like(inp)
    with pytest.raises(CError, match="Unsupported data type"):
        uniform_weights(uvw.astype(np.float32), freqs, mx, grid, inp, out)
    with pytest.raises(CError, match="Unsupported data type"):
        uniform_weights(uvw, freqs, mx, grid.astype(np.float32), inp, out)
    with pytest.raises(CError, match="Generic runtime error"):
        uniform_weights(uvw, freqs, mx, grid, inp[0], out[0])
    with pytest.raises(CError):
        uniform_weights(uvw, freqs, mx, np.zeros((3, 4, 1)), inp, out)
    import torch
    with pytest.raises(CError, match="Memory location"):
        uniform_weights(uvw, freqs, mx, torch.zeros((3, 3, 1),
                        dtype=torch.float64, device=device), inp, out)
    # A host input_weight with device outputs is a location error, never a
    # host pointer handed to a kernel.
    d = [torch.from_numpy(a).to(device) for a in (uvw, freqs, grid, out)]
    with pytest.raises(CError, match="Memory location"):
        uniform_weights(d[0], d[1], mx, d[2], inp, d[3])
    # An input smaller than the output is rejected, not read past its end.
    small = torch.from_numpy(np.ascontiguousarray(inp[:, :, :1])).to(device)
    with pytest.raises(CError):
        uniform_weights(d[0], d[1], mx, d[2], small, d[3])
