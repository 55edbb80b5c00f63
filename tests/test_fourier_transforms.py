"""sdp_fft / sdp_pswf / sdp_fft_padded_size: the drop-in FFT and PSWF ABI.

CPU tests (host-side functions):
  * PSWF values equal the reference's own golden vectors
    (tests/fourier_transforms/test_pswf.cpp:123-162 of the reference:
    PSWF(0, 8) and PSWF(1, 12) on 16 points, PSWF(0, 4) on 32 points) to
    the reference's tolerances (6e-13 relative in double, 6e-8 in float);
  * sdp_fft_padded_size equals a restatement of the reference's min-heap
    walk (sdp_fft_padded_size.cpp:87-126) for every n up to 5000.
GPU tests: the reference's test_fft.py cases (numpy.fft, assert_allclose
defaults) on host and device arrays, plus 3-D, exec_shift, norm, phase and
the argument checks of sdp_fft.cpp:295-356.
"""
import heapq
import math

import numpy as np
import pytest

# tests/fourier_transforms/test_pswf.cpp:123-162 of the reference.
REF_0_8_16 = [
    0., 0.027739141134746, 0.091191127759381,
    0.209044784141754, 0.382566549867655, 0.5914940612484,
    0.795355148039012, 0.944953307469797, 0.999999999999999,
    0.944953307469797, 0.795355148039012, 0.5914940612484,
    0.382566549867655, 0.209044784141754, 0.091191127759381,
    0.027739141134746]
REF_1_12_16 = [
    0., 0.003294739717825, 0.02282344776114,
    0.085481700400665, 0.221815527395368, 0.439706432303182,
    0.699133301246467, 0.915341842238297, 0.999999999999999,
    0.915341842238297, 0.699133301246467, 0.439706432303182,
    0.221815527395368, 0.085481700400665, 0.02282344776114,
    0.003294739717825]
REF_0_4_32 = [
    0., 0.170790162306119, 0.229028505587468,
    0.293249007653473, 0.362375107129104, 0.435092139714442,
    0.509883171680941, 0.585074290491016, 0.658887707928077,
    0.729500645949425, 0.795107677241523, 0.853983996619878,
    0.904547016598184, 0.94541371587235, 0.975451322633679,
    0.99381917932372, 1., 0.99381917932372,
    0.975451322633679, 0.94541371587235, 0.904547016598184,
    0.853983996619878, 0.795107677241523, 0.729500645949425,
    0.658887707928077, 0.585074290491016, 0.509883171680941,
    0.435092139714442, 0.362375107129104, 0.293249007653473,
    0.229028505587468, 0.170790162306119]


@pytest.mark.parametrize("m,c,ref", [(0, 8.0, REF_0_8_16),
                                     (1, 12.0, REF_1_12_16),
                                     (0, 4.0, REF_0_4_32)])
@pytest.mark.parametrize("dtype,limit", [(np.float64, 6e-13),
                                         (np.float32, 6e-8),
                                         (np.complex128, 6e-13),
                                         (np.complex64, 6e-8)])
def test_generate_pswf_matches_reference_golden(m, c, ref, dtype, limit):
    from ska_sdp_func.fourier_transforms import generate_pswf

    out = np.zeros(len(ref), dtype)
    generate_pswf(m, c, out)
    expected = np.array(ref)
    scale = np.maximum(expected, 1e-15)
    # test_pswf.cpp:72-76
    assert np.all(np.abs(out.real - expected) / scale < limit)


def test_pswf_plan_api():
    from ska_sdp_func.fourier_transforms import Pswf, generate_pswf

    p = Pswf(0, 8.0)
    assert p.c == 8.0 and p.m == 0
    assert p.evaluate(1.0) == 0.0 and p.evaluate(-1.5) == 0.0
    ref = np.zeros(16)
    generate_pswf(0, 8.0, ref)
    for i in range(1, 8):
        assert abs(p.evaluate(2 * i / 16) - ref[8 + i]) < 1e-15
        assert p.evaluate(-2 * i / 16) == p.evaluate(2 * i / 16)
    out = np.zeros(16, np.float32)
    p.generate(out, 0, True)
    assert out[0] == np.float32(1e-15)
    # m = 2: Flammer normalisation S_22(c, 0) = P_2^2(0) = 3.
    assert abs(Pswf(2, 5.0).evaluate(0.0) - 3.0) < 1e-12


@pytest.mark.parametrize("m", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("c", [1.0, 2.5, 5.0, 8.0, 12.0, 20.0])
def test_pswf_matches_specfun_all_orders(m, c):
    """S_mm(c, x) for m >= 2 and x != 0 as well: scipy.special.pro_ang1 is
    Zhang & Jin's specfun (SDMN / SCKB / ASWFA), the routines the reference
    sdp_pswf.cpp:27-564 restates, so it stands in for the reference at every
    order; agreement 1e-14 relative (c <= 12) and 1e-11 at c = 20, where
    specfun's own power series loses digits."""
    import scipy.special as sp
    from ska_sdp_func.fourier_transforms import Pswf

    p = Pswf(m, c)
    xs = np.linspace(-0.98, 0.98, 41)
    got = np.array([p.evaluate(x) for x in xs])
    ref = np.array([sp.pro_ang1(m, m, c, abs(x))[0] for x in xs])
    tol = 1e-14 if c <= 12 else 1e-11
    assert np.max(np.abs(got - ref)) <= tol * np.max(np.abs(ref))


def _padded_size_heap(n, padding_factor):
    """Restatement of sdp_fft_padded_size.cpp:87-126 (min-heap walk)."""
    heap = [2]
    prev = 0
    n = int(math.ceil(n * padding_factor))
    limit = 2 * n
    nxt = 0
    while heap:
        nxt = heapq.heappop(heap)
        if nxt >= n:
            break
        if nxt == prev:
            continue
        prev = nxt
        for p in (2, 3, 5, 7, 11):
            if nxt * p <= limit:
                heapq.heappush(heap, nxt * p)
    return nxt


def test_padded_size_matches_reference_algorithm():
    from ska_sdp_func.fourier_transforms import padded_fft_size

    for n in range(0, 5001):
        assert padded_fft_size(n, 1.0) == _padded_size_heap(n, 1.0), n
    for n, f in [(256, 1.2), (1000, 1.1), (4097, 1.5), (333, 2.0)]:
        assert padded_fft_size(n, f) == _padded_size_heap(n, f)


# ----------------------------------------------------------------- GPU ----

def _fft(inp, out, nd, fwd):
    from ska_sdp_func.fourier_transforms import Fft

    f = Fft(inp, out, nd, fwd)
    f.exec(inp, out)
    return f


def _rand(rng, shape, dtype=np.complex128):
    return (rng.random(shape) + 1j * rng.random(shape)).astype(dtype)


@pytest.mark.gpu
@pytest.mark.parametrize("on_device", [False, True])
def test_reference_fft_cases(device, on_device):
    """tests/fourier_transforms/test_fft.py:15-146 of the reference."""
    import torch

    rng = np.random.default_rng(1)
    dev = (lambda a: torch.from_numpy(a).to(device)) if on_device else \
        (lambda a: a.copy())
    back = (lambda t: t.cpu().numpy()) if on_device else (lambda a: a)
    # 1-D
    x = rng.random(256) + 0j
    i, o = dev(x), dev(np.zeros_like(x))
    _fft(i, o, 1, True)
    np.testing.assert_allclose(back(o), np.fft.fft(x))
    # 2-D of ones
    x = np.ones((256, 256)) + 0j
    i, o = dev(x), dev(np.zeros_like(x))
    _fft(i, o, 2, True)
    np.testing.assert_allclose(back(o), np.fft.fft2(x), atol=1e-9)
    assert back(o)[0, 0] == x.size
    # 2-D, forward and inverse
    x = _rand(rng, (256, 512))
    i, o = dev(x), dev(np.zeros_like(x))
    _fft(i, o, 2, True)
    np.testing.assert_allclose(back(o), np.fft.fft2(x))
    i, o = dev(x), dev(np.zeros_like(x))
    _fft(i, o, 2, False)
    np.testing.assert_allclose(back(o) / x.size, np.fft.ifft2(x))
    # stack of 2-D transforms (batch = first dimension)
    x = _rand(rng, (4, 256, 512))
    i, o = dev(x), dev(np.zeros_like(x))
    _fft(i, o, 2, True)
    np.testing.assert_allclose(back(o), np.fft.fft2(x, axes=(1, 2)))


@pytest.mark.gpu
def test_fft_single_precision_3d_and_in_place(device):
    import torch

    rng = np.random.default_rng(2)
    x = _rand(rng, (32, 48, 64), np.complex64)
    t = torch.from_numpy(x).to(device)
    o = torch.zeros_like(t)
    _fft(t, o, 3, True)
    ref = np.fft.fftn(x.astype(np.complex128))
    err = np.linalg.norm(o.cpu().numpy() - ref) / np.linalg.norm(ref)
    assert err < 1e-6
    # in place, batched 1-D inverse
    y = _rand(rng, (7, 1000), np.complex64)
    t = torch.from_numpy(y).to(device)
    _fft(t, t, 1, False)
    ref = np.fft.ifft(y.astype(np.complex128), axis=1) * 1000
    err = np.linalg.norm(t.cpu().numpy() - ref) / np.linalg.norm(ref)
    assert err < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.complex128, np.complex64])
def test_exec_shift_norm_phase(device, dtype):
    import torch
    from ska_sdp_func.fourier_transforms import Fft
    from ska_sdp_func.fourier_transforms.fft import fft_norm, fft_phase

    rng = np.random.default_rng(3)
    x = _rand(rng, (128, 96), dtype)
    t = torch.from_numpy(x).to(device)
    f = Fft(t, t, 2, False)
    f.exec_shift(t, norm=True)
    # phase . ifft . phase with 1 / N = fftshift(ifft2(ifftshift)) for
    # even sizes
    ref = np.fft.fftshift(np.fft.ifft2(np.fft.ifftshift(
        x.astype(np.complex128))))
    tol = 1e-12 if dtype == np.complex128 else 2e-6
    err = np.linalg.norm(t.cpu().numpy() - ref) / np.linalg.norm(ref)
    assert err < tol
    h = x.copy()
    fft_phase(h)
    sgn = np.where((np.add.outer(np.arange(128), np.arange(96)) & 1) == 1,
                   -1, 1)
    assert np.array_equal(h, x * sgn)
    h = x.copy()
    fft_norm(h)
    np.testing.assert_allclose(h, x * (1.0 / x.size), rtol=1e-6)


@pytest.mark.gpu
def test_fft_argument_checks(device):
    import torch
    from ska_sdp_func.fourier_transforms import Fft
    from ska_sdp_func.utility import CError

    a = np.zeros((16, 16), np.complex128)
    with pytest.raises(CError, match="Error 3"):     # data type
        Fft(np.zeros((16, 16)), np.zeros((16, 16)), 2, True)
    with pytest.raises(CError, match="Error 6"):     # location
        Fft(a, torch.zeros((16, 16), dtype=torch.complex128,
                           device=device), 2, True)
    with pytest.raises(CError, match="Error 1"):     # dimensions
        Fft(a, np.zeros((16, 8), np.complex128), 2, True)
    with pytest.raises(CError, match="Error 1"):     # FFT rank
        Fft(a, a.copy(), 3, True)
    with pytest.raises(CError, match="Error 1"):     # read-only output
        ro = a.copy()
        ro.flags.writeable = False
        Fft(a, ro, 2, True)
    f = Fft(a, a.copy(), 2, True)
    with pytest.raises(CError, match="Error 1"):     # not the plan's arrays
        f.exec(np.zeros((8, 8), np.complex128), np.zeros((8, 8),
                                                         np.complex128))
