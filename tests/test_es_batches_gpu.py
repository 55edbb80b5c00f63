"""Calls larger than one bucketing batch (sdp_gridder_uvw_es_fft.hip,
batch_vis_limit): the call is split into row batches whose tiles are added
into one grid (gridding) or gathered from one transformed grid
(degridding), so bucketing record indices stay 32-bit and the record
scratch bounded.

* small cases with the cap lowered (set_max_batch) against the oracle and
  against the unbatched call: 2-D / 3-D, f32 / f64, grid / degrid, the
  split scatter API, a cap that leaves a one-row last batch;
* a call of 17M rows x 64 channels = 1.09e9 visibilities (> 2^30, beyond
  the 32-bit entry range of a single bucketing) with the default cap:
  the dirty image equals the sum of the images of its two halves and the
  degridded visibilities equal those of the halves, to f32 rounding.
Tolerances: relative L2 1e-5 (f32) / 1e-12 (f64) against the oracle, as
tests/test_es_gpu.py; batched vs unbatched differ by summation order only.
"""
import numpy as np
import pytest

from es_data import make_case, rel_l2
from oracle import es_oracle

pytestmark = pytest.mark.gpu


def _gpu(x, device):
    import torch

    return torch.from_numpy(np.ascontiguousarray(x)).to(device)


def _plan(g, px, eps, do_w, cap):
    from ska_sdp_func.grid_data import GridderUvwEsFft

    plan = GridderUvwEsFft(*g, px, px, eps, do_w)
    plan.set_max_batch(cap)
    return plan


@pytest.mark.parametrize("dbl,do_w,rows,chan,cap", [
    (False, False, 30000, 3, 20000),
    (False, False, 2001, 3, 303),   # 101-row batches, the last of 82 rows
    (False, True, 12000, 2, 9000),
    (True, False, 9000, 3, 10000),
    (True, True, 5000, 2, 4000),
])
def test_batched_grid_and_degrid_match_oracle(device, dbl, do_w, rows, chan,
                                              cap):
    import torch

    eps = 1e-12 if dbl else 1e-5
    tol = 1e-12 if dbl else 1e-5
    n = 256
    uvw, freq, vis, wt, px = make_case(11, rows, chan, n, dbl=dbl,
                                       w_range=200.0)
    rdt = np.float64 if dbl else np.float32
    dirty0 = np.zeros((n, n), rdt)
    g = [_gpu(a, device) for a in (uvw, freq, vis, wt, dirty0)]
    plan = _plan(g, px, eps, do_w, cap)
    assert plan.batch_vis == cap
    assert rows * chan > cap
    plan.grid_uvw_es_fft(*g)
    got = g[4].cpu().numpy()
    geo = es_oracle.geometry_for(uvw, freq, vis, dirty0, px, eps, do_w)
    ref = es_oracle.grid_uvw_es_fft(geo, uvw, freq, vis, wt, dirty0)
    assert rel_l2(got, ref) <= tol

    # The unbatched call of the same plan agrees to summation order.
    plan.set_max_batch(0)
    g[4].zero_()
    plan.grid_uvw_es_fft(*g)
    assert rel_l2(got, g[4].cpu().numpy()) <= (1e-13 if dbl else 1e-6)

    image = np.random.default_rng(5).standard_normal((n, n)).astype(rdt)
    ref_vis, _ = es_oracle.ifft_degrid_uvw_es(geo, uvw, freq, image)
    plan.set_max_batch(cap)
    g[4].copy_(_gpu(image, device))
    out = torch.zeros_like(g[2])
    plan.ifft_grid_uvw_es(g[0], g[1], out, g[3], g[4])
    assert rel_l2(out.cpu().numpy(), ref_vis) <= tol


def test_batched_split_scatter(device):
    """The multi-GPU split API in batches: scatter into a caller grid (which
    the batched form zeroes first), finish, equal to the whole call."""
    import torch

    n = 256
    uvw, freq, vis, wt, px = make_case(12, 40000, 2, n)
    dirty0 = np.zeros((n, n), np.float32)
    g = [_gpu(a, device) for a in (uvw, freq, vis, wt, dirty0)]
    plan = _plan(g, px, 1e-5, False, 25000)
    G = plan.grid_size
    grid = torch.full((G, G), 7.0, dtype=torch.complex64, device=device)
    plan.grid_scatter(g[0], g[1], g[2], g[3], grid)
    plan.grid_finish(grid, g[4])
    geo = es_oracle.geometry_for(uvw, freq, vis, dirty0, px, 1e-5, False)
    ref = es_oracle.grid_uvw_es_fft(geo, uvw, freq, vis, wt, dirty0)
    assert rel_l2(g[4].cpu().numpy(), ref) <= 1e-5


def test_channels_beyond_one_batch_rejected(device):
    from ska_sdp_func.utility import CError

    n = 128
    uvw, freq, vis, wt, px = make_case(13, 100, 8, n)
    g = [_gpu(a, device) for a in (uvw, freq, vis, wt,
                                    np.zeros((n, n), np.float32))]
    plan = _plan(g, px, 1e-5, False, 4)
    with pytest.raises(CError, match="Error 2"):
        plan.grid_uvw_es_fft(*g)


def test_call_past_2_30_visibilities_equals_sum_of_halves(device):
    """17M rows x 64 channels = 1.088e9 visibilities > 2^30 in one call
    (config-3 distribution, 1.0-1.49 GHz), default batch cap. Beside the
    sum-of-halves checks (the batching is invisible), parity: degridded
    visibilities of sampled rows from the start, the middle and the end of
    the call (flat indices up to 1.088e9, past 2^30 and in the last row
    batch) against the oracle, and gridding tied to that degridding over
    all 1.088e9 visibilities by the adjoint identity the reference's own
    test uses, <grid(V), I> = Re<V, degrid(I)>."""
    import torch
    from ska_sdp_func.grid_data import GridderUvwEsFft

    R, C, n = 17_000_000, 64, 5440
    assert R * C > 2 ** 30
    px = 2.0 * np.pi / 180.0 / n
    gen = torch.Generator(device=device)
    gen.manual_seed(20251015 + 30)
    freq = (1e9 + torch.arange(C, device=device, dtype=torch.float64)
            * (0.5e9 / C)).to(torch.float32)
    umax = 0.45 * 299792458.0 / (float(freq[-1]) * px)
    r = umax * torch.sqrt(torch.rand(R, generator=gen, device=device))
    th = 2 * np.pi * torch.rand(R, generator=gen, device=device)
    w = (torch.rand(R, generator=gen, device=device) - 0.5) * 1000.0
    uvw = torch.stack([r * torch.cos(th), r * torch.sin(th), w], 1).contiguous()
    del r, th, w
    vis = torch.complex(torch.randn((R, C), generator=gen, device=device),
                        torch.randn((R, C), generator=gen, device=device))
    wt = torch.ones((R, C), dtype=torch.float32, device=device)
    dirty = torch.zeros((n, n), dtype=torch.float32, device=device)
    plan = GridderUvwEsFft(uvw, freq, vis, wt, dirty, px, px, 1e-5, False)
    assert plan.batch_vis < 2 ** 30
    plan.grid_uvw_es_fft(uvw, freq, vis, wt, dirty)
    h = R // 2
    halves = torch.zeros_like(dirty)
    for a, b in ((0, h), (h, R)):
        part = torch.zeros_like(dirty)
        plan.grid_uvw_es_fft(uvw[a:b].contiguous(), freq,
                             vis[a:b].contiguous(), wt[a:b].contiguous(), part)
        halves += part
    torch.cuda.synchronize()
    err = float(torch.linalg.norm((dirty - halves).double())
                / torch.linalg.norm(halves.double()))
    print(f"> 2^30 visibilities: grid vs sum of halves rel-L2 {err:.2e}")
    assert err <= 1e-5
    assert float(torch.linalg.norm(dirty.double())) > 0

    image = torch.randn((n, n), generator=gen, device=device)
    out = torch.zeros_like(vis)
    img = image.clone()
    plan.ifft_grid_uvw_es(uvw, freq, out, wt, img)
    parts = []
    for a, b in ((0, h), (h, R)):
        o = torch.zeros((b - a, C), dtype=torch.complex64, device=device)
        img = image.clone()
        plan.ifft_grid_uvw_es(uvw[a:b].contiguous(), freq, o, wt[a:b], img)
        parts.append(o)
    ref = torch.cat(parts)
    err = float(torch.linalg.norm(out - ref) / torch.linalg.norm(ref))
    print(f"> 2^30 visibilities: degrid vs halves rel-L2 {err:.2e}")
    assert err <= 1e-6
    assert int((out == 0).sum()) == 0
    del parts, ref

    rows = np.concatenate([np.arange(0, 64), np.arange(h - 32, h + 32),
                           np.arange(R - 128, R)])
    assert (rows[-1] + 1) * C > 2 ** 30
    uvw_s = uvw[rows].cpu().numpy()
    f_np = freq.cpu().numpy()
    img_np = image.cpu().numpy()
    geo = es_oracle.geometry_for(uvw_s, f_np, vis[rows].cpu().numpy(),
                                 img_np, px, 1e-5, False)
    ref_s, _ = es_oracle.ifft_degrid_uvw_es(geo, uvw_s, f_np, img_np)
    err = rel_l2(out[rows].cpu().numpy(), ref_s)
    print(f"> 2^30 visibilities: sampled degrid vs oracle rel-L2 {err:.2e}")
    assert err <= 1e-5

    adj1 = float((dirty.double() * image.double()).sum())
    adj2 = 0.0
    step = 1 << 20
    for a in range(0, R, step):
        o, v = out[a:a + step], vis[a:a + step]
        adj2 += float((o.real.double() * v.real.double()
                       + o.imag.double() * v.imag.double()).sum())
    adj_err = abs(adj1 - adj2) / max(abs(adj1), abs(adj2))
    print(f"> 2^30 visibilities: adjoint identity error {adj_err:.2e}")
    assert adj_err < 1e-5
