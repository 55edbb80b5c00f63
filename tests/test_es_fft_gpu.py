"""GPU parity of the pruned, fused FFT passes (csrc/grid_data/es_fft.hip).

f32 plans on power-of-two grids (1024..16384) replace rocFFT + the separate
screen / correction kernels by three fused passes. Checked here:
  * against the CPU oracle (float64 FFT of the full grid, then crop) for
    G = 1024, 2048, 4096, 2-D and 3-D, even and odd image sizes, both
    directions -- relative L2 < 1e-5 (the f32 parity bound);
  * against this library's own rocFFT path (SDP_ES_FFT=rocfft) at the
    benchmark geometry (G = 8192, N = 5440, 2-D) and at G = 16384 --
    relative L2 < 2e-6 (the same geometries against the oracle itself:
    tests/test_baseline_configs_gpu.py, 3-D at G = 8192 included);
  * the split scatter/finish API and odd-N untouched last row/column;
  * the w-towers plane transform (whole-grid FFT in place with permuted
    output rows, sdp_fft_2d_inplace_permuted) at G = 1024 and 16384 against
    scipy.fft in float64, both directions -- relative L2 < 1e-5.
2-D plans with 2048 <= G <= 8192 take the real-output (gridding) and
real-input (degridding) forms of the transform (half-length column passes);
the cases above at G = 2048, 4096 and 8192 cover them, odd N included.
"""
import os

import numpy as np
import pytest

from es_data import make_case, rel_l2
from oracle import es_oracle

pytestmark = pytest.mark.gpu


def _gpu(x, device):
    import torch

    return torch.from_numpy(np.ascontiguousarray(x)).to(device)


def _plan(g, px, eps, do_w, rocfft=False):
    from ska_sdp_func.grid_data import GridderUvwEsFft

    old = os.environ.pop("SDP_ES_FFT", None)
    if rocfft:
        os.environ["SDP_ES_FFT"] = "rocfft"
    try:
        plan = GridderUvwEsFft(*g, px, px, eps, do_w)
    finally:
        os.environ.pop("SDP_ES_FFT", None)
        if old is not None:
            os.environ["SDP_ES_FFT"] = old
    return plan


def _grid(device, case, dirty0, eps, do_w, rocfft=False):
    uvw, freq, vis, wt, px = case
    g = [_gpu(a, device) for a in (uvw, freq, vis, wt, dirty0)]
    plan = _plan(g, px, eps, do_w, rocfft)
    plan.grid_uvw_es_fft(*g)
    return g[4].cpu().numpy(), plan


def _degrid(device, case, dirty, eps, do_w, rocfft=False):
    uvw, freq, vis, wt, px = case
    g = [_gpu(a, device) for a in (uvw, freq, np.zeros_like(vis), wt, dirty)]
    plan = _plan(g, px, eps, do_w, rocfft)
    plan.ifft_grid_uvw_es(*g)
    return g[2].cpu().numpy(), g[4].cpu().numpy(), plan


ORACLE_CASES = [
    # (N, do_w, eps) -> G
    (680, False, 1e-5),    # 1024
    (673, False, 1e-5),    # 1024, odd N
    (840, False, 0.05),    # 1024, config-1 kernel (W = 4)
    (1360, False, 1e-5),   # 2048
    (1349, True, 1e-5),    # 2048, odd N, w-stacking
    (1349, False, 1e-5),   # 2048, odd N, 2-D (real-output / real-input form)
    (2701, False, 1e-5),   # 4096, odd N, 2-D
    (680, True, 1e-5),     # 1024, w-stacking
    (2720, False, 1e-5),   # 4096
]


@pytest.mark.parametrize("n,do_w,eps", ORACLE_CASES)
def test_fused_grid_matches_oracle(device, n, do_w, eps):
    case = make_case(21, 6000, 2, n, w_range=200.0)
    dirty0 = np.random.default_rng(1).standard_normal((n, n)).astype(np.float32)
    out, plan = _grid(device, case, dirty0, eps, do_w)
    assert plan.fused_fft
    geo = es_oracle.geometry_for(case[0], case[1], case[2], dirty0, case[4],
                                 eps, do_w)
    assert plan.grid_size == geo["grid_size"]
    ref = es_oracle.grid_uvw_es_fft(geo, case[0], case[1], case[2], case[3],
                                    dirty0)
    assert rel_l2(out, ref) < 1e-5
    if n % 2:
        # odd N: the last row / column is never written (reference quirk)
        assert np.array_equal(out[-1, :], dirty0[-1, :])
        assert np.array_equal(out[:, -1], dirty0[:, -1])


@pytest.mark.parametrize("n,do_w,eps", ORACLE_CASES)
def test_fused_degrid_matches_oracle(device, n, do_w, eps):
    case = make_case(22, 6000, 2, n, w_range=200.0)
    dirty = np.random.default_rng(2).standard_normal((n, n)).astype(np.float32)
    out_vis, out_dirty, plan = _degrid(device, case, dirty, eps, do_w)
    assert plan.fused_fft
    geo = es_oracle.geometry_for(case[0], case[1], case[2], dirty, case[4],
                                 eps, do_w)
    ref_vis, ref_dirty = es_oracle.ifft_degrid_uvw_es(geo, case[0], case[1],
                                                      dirty)
    assert rel_l2(out_vis, ref_vis) < 1e-5
    assert rel_l2(out_dirty, ref_dirty) < 1e-6
    if n % 2:
        assert np.array_equal(out_dirty[-1, :], dirty[-1, :])


@pytest.mark.parametrize("n,do_w", [(5440, False), (5403, False)])
def test_fused_matches_rocfft_config2_geometry(device, n, do_w):
    case = make_case(23, 200000, 1, n, w_range=300.0)
    dirty0 = np.random.default_rng(3).standard_normal((n, n)).astype(np.float32)
    a, pa = _grid(device, case, dirty0, 1e-5, do_w)
    b, pb = _grid(device, case, dirty0, 1e-5, do_w, rocfft=True)
    assert pa.grid_size == 8192 and pa.fused_fft and not pb.fused_fft
    assert rel_l2(a, b) < 2e-6
    va, da, _ = _degrid(device, case, dirty0, 1e-5, do_w)
    vb, db, _ = _degrid(device, case, dirty0, 1e-5, do_w, rocfft=True)
    assert rel_l2(va, vb) < 2e-6
    assert np.array_equal(da, db)


def test_fused_matches_rocfft_16384(device):
    n = 10800
    case = make_case(24, 50000, 1, n)
    dirty0 = np.zeros((n, n), np.float32)
    a, pa = _grid(device, case, dirty0, 1e-5, False)
    b, _ = _grid(device, case, dirty0, 1e-5, False, rocfft=True)
    assert pa.grid_size == 16384 and pa.fused_fft
    assert rel_l2(a, b) < 2e-6
    d = np.random.default_rng(4).standard_normal((n, n)).astype(np.float32)
    va, _, _ = _degrid(device, case, d, 1e-5, False)
    vb, _, _ = _degrid(device, case, d, 1e-5, False, rocfft=True)
    assert rel_l2(va, vb) < 2e-6


def test_fused_split_scatter_finish_equals_grid(device):
    import torch

    n = 680
    uvw, freq, vis, wt, px = make_case(25, 4000, 2, n)
    g = [_gpu(a, device) for a in (uvw, freq, vis, wt)]
    d1 = torch.zeros((n, n), dtype=torch.float32, device=device)
    d2 = torch.zeros_like(d1)
    plan = _plan(g + [d1], px, 1e-5, False)
    assert plan.fused_fft
    plan.grid_uvw_es_fft(*g, d1)
    G = plan.grid_size
    half = len(uvw) // 2
    total = torch.zeros((G, G), dtype=torch.complex64, device=device)
    for sl in (slice(0, half), slice(half, None)):
        gr = torch.empty((G, G), dtype=torch.complex64, device=device)
        plan.grid_scatter(g[0][sl].contiguous(), g[1], g[2][sl].contiguous(),
                          g[3][sl].contiguous(), gr)
        total += gr
    plan.grid_finish(total, d2)
    torch.cuda.synchronize()
    assert rel_l2(d2.cpu().numpy(), d1.cpu().numpy()) < 1e-6


@pytest.mark.parametrize("G", [1024, 16384])
@pytest.mark.parametrize("forward", [True, False])
def test_plane_fft_permuted_vs_numpy(device, G, forward):
    """The w-stack plane transform (sdp_fft_2d_inplace_permuted, the fused
    three-pass FFT the w-towers image side runs in place) against
    scipy.fft in float64, output rows read through the permutation."""
    import scipy.fft
    import torch
    from ska_sdp_func.fourier_transforms import (fft_2d_inplace_permuted,
                                                 fft_permuted_n2)

    gen = torch.Generator(device=device)
    gen.manual_seed(G + forward)
    x = torch.complex(torch.randn((G, G), generator=gen, device=device),
                      torch.randn((G, G), generator=gen, device=device))
    host = x.cpu().numpy().astype(np.complex128)
    fft_2d_inplace_permuted(x, forward)
    n2 = fft_permuted_n2(G)
    n1 = G // n2
    k = np.arange(G)
    got = x.cpu().numpy()[n1 * (k % n2) + k // n2]
    del x
    if forward:
        ref = scipy.fft.fft2(host, workers=8)
    else:
        ref = scipy.fft.ifft2(host, norm="forward", workers=8)
    del host
    err = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
    print(f"plane FFT G {G} forward {forward}: rel-L2 {err:.2e}")
    assert err < 1e-5


def test_plane_fft_twiddles_per_device(device):
    """The permuted plane FFT keeps its twiddle tables per (device, G): a
    transform on a second GPU after one on the first must use tables in its
    own memory (advisor finding, round 5). Runs on every visible device in
    turn, against numpy; with one GPU it checks the per-device key on
    device 0 twice."""
    import torch
    from ska_sdp_func.fourier_transforms import (fft_2d_inplace_permuted,
                                                 fft_permuted_n2)

    G = 1024
    n2 = fft_permuted_n2(G)
    k = np.arange(G)
    rng = np.random.default_rng(11)
    host = (rng.standard_normal((G, G)) + 1j * rng.standard_normal((G, G)))
    ref = np.fft.fft2(host)
    devs = list(range(torch.cuda.device_count())) or [0]
    for d in devs + devs[:1]:
        with torch.cuda.device(d):
            x = torch.from_numpy(host.astype(np.complex64)).to(f"cuda:{d}")
            fft_2d_inplace_permuted(x, True)
            got = x.cpu().numpy()[(G // n2) * (k % n2) + k // n2]
        err = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
        assert err < 1e-5, (d, err)
