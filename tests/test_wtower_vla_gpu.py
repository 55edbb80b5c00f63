"""The reference's own w-stacking x w-towers accuracy test, on the GPU.

Recipe of tests/grid_data/test_gridder_wtower_uvw.cpp of ska-sdp-func
1.2.2 (:264-330 layout, :408-649 run_and_check and main): the 27-antenna
VLA layout tracked for 16 hour angles over 90 degrees at declination 40
degrees (5616 rows), 2 channels at f0 = c, df = c / 100, a 512^2 model of
four point sources at 3.2 arcsec cells, padded to 2 * sdp_fft_padded_size(
256, 1.2) = 616 pixels; sub-grid 256, W = W_w = 8, oversampling 16384,
sub-grid fraction 2/3, w_step and w-tower height from the library's own
determine_w_step / determine_max_w_tower_height. Reference data by direct
Fourier transforms through the library's sdp_gridder_dft / _idft (as the
reference test does), cross-checked here against the numpy restatement
(oracle/wtower_oracle.py). Thresholds of the reference: RMS difference of
the degridded visibilities and of the gridded, trimmed image < 1e-3
(:505, :539).

The reference runs the CPU and GPU variants of three type combinations
(uvw f64 / vis c128, uvw f64 / vis c64, uvw f32 / vis c64), all with a
complex-double image; host ("CPU") arrays are staged through the GPU
here, so both locations exercise the HIP kernels. One more case puts a
complex-float image on a power-of-two 1024^2 grid, the configuration that
takes the fused towers and the fused in-place plane FFT of
csrc/grid_data/es_fft.hip (fft2d_inplace_permuted).
"""
import math

import numpy as np
import pytest

from oracle import wtower_oracle as wo

pytestmark = pytest.mark.gpu

C_0 = 299792458.0
CELL_ARCSEC = 3.2
FREQ0, DFREQ = C_0, C_0 / 100
IMAGE_SIZE, NUM_CHAN, SUBGRID = 512, 2, 256

# VLA antenna (x, y, z) coordinates [m] of the reference test
# (test_gridder_wtower_uvw.cpp:268-296).
VLA_XYZ = np.array([
    [-401.2842, -270.6395, 1.3345],
    [-1317.9926, -889.0279, 2.0336],
    [-2642.9943, -1782.7459, 7.8328],
    [-4329.9414, -2920.6298, 4.217],
    [-6350.012, -4283.1247, -6.0779],
    [-8682.4872, -5856.4585, -7.3861],
    [-11311.4962, -7629.385, -19.3219],
    [-14224.3397, -9594.0268, -32.2199],
    [-17410.1952, -11742.6658, -52.5716],
    [438.6953, -204.4971, -0.1949],
    [1440.9974, -671.8529, 0.6199],
    [2889.4597, -1347.2324, 12.4453],
    [4733.627, -2207.126, 19.9349],
    [6942.0661, -3236.8423, 28.0543],
    [9491.9269, -4425.5098, 19.3104],
    [12366.0731, -5765.3061, 13.8351],
    [15550.4596, -7249.6904, 25.3408],
    [19090.2771, -8748.4418, -53.2768],
    [-38.0377, 434.7135, -0.026],
    [-124.9775, 1428.1567, -1.4012],
    [-259.3684, 2963.3547, -0.0815],
    [-410.6587, 4691.5051, -0.3722],
    [-602.292, 6880.1408, 0.5885],
    [-823.5569, 9407.5172, 0.0647],
    [-1072.9272, 12255.8935, -4.2741],
    [-1349.2489, 15411.7447, -7.7693],
    [-1651.4637, 18863.4683, -9.2248],
])


def vla_uvw(num_times=16, dec_deg=40.0):
    """xyz_to_uvw + calculate_baselines (test :35-86, :300-330)."""
    dec = math.radians(dec_deg)
    out = []
    x, y, z = VLA_XYZ.T
    for t in range(num_times):
        ha = t * (math.pi / 2.0) / num_times
        v0 = x * math.sin(ha) + y * math.cos(ha)
        ant = np.stack([x * math.cos(ha) - y * math.sin(ha),
                        z * math.cos(dec) + v0 * math.sin(dec),
                        z * math.sin(dec) - v0 * math.cos(dec)], axis=1)
        i, j = np.triu_indices(len(ant), 1)
        out.append(ant[j] - ant[i])
    return np.concatenate(out)


def model_image(size=IMAGE_SIZE):
    """generate_model_image (test :121-150)."""
    img = np.zeros((size, size), np.complex128)
    h = size // 2
    img[h + size // 4, h + 2] = 2
    img[h - size // 4 + 2, h + size // 4 - 12] = 1
    img[h - size // 3 - 12, h - size // 4 - 12] = 1.6
    img[h - 12, h - size // 3 - 12] = 2.3
    return img


@pytest.fixture(scope="module")
def reference(device):
    """Reference visibilities and image by DFT (test :616-648), through the
    library, each checked against the numpy restatement."""
    import torch
    import ska_sdp_func.grid_data as g

    cell = math.radians(CELL_ARCSEC / 3600.0)
    fov = math.sin(cell) * IMAGE_SIZE
    model = model_image()
    uvw = vla_uvw()
    rows = len(uvw)
    nsrc = g.count_nonzero_pixels(model)
    assert nsrc == 4
    flux = np.zeros(nsrc)
    lmn = np.zeros((nsrc, 3))
    g.image_to_flmn(model, fov, 0.0, 0.0, None, flux, lmn)
    rf, rl = wo.image_to_flmn(model, fov, 0.0, 0.0)
    np.testing.assert_array_equal(flux, rf)
    np.testing.assert_array_equal(lmn, rl)
    ref_vis = np.zeros((rows, NUM_CHAN), np.complex128)
    g.dft(uvw, None, None, flux, lmn, 0, 0, 0, fov, 0.0, FREQ0, DFREQ,
          ref_vis)
    chk = wo.dft_vis(uvw, None, None, flux, lmn, 0, 0, 0, fov, 0.0, FREQ0,
                     DFREQ, np.zeros_like(ref_vis))
    assert np.max(np.abs(ref_vis - chk)) < 1e-10
    lmn_all = np.zeros((IMAGE_SIZE * IMAGE_SIZE, 3))
    g.image_to_flmn(model, fov, 0.0, 0.0, None, None, lmn_all)
    img = torch.zeros((IMAGE_SIZE, IMAGE_SIZE), dtype=torch.complex128,
                      device=device)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
    g.idft(dev(uvw), dev(ref_vis), None, None, dev(lmn_all), None, 0, 0, 0,
           fov, 0.0, FREQ0, DFREQ, img)
    ref_img = img.cpu().numpy() / (rows * NUM_CHAN)
    # numpy check of the library iDFT at sampled pixels
    sel = np.random.default_rng(0).choice(IMAGE_SIZE ** 2, 1500,
                                          replace=False)
    u = uvw[:, 0:1] * (FREQ0 + DFREQ * np.arange(NUM_CHAN)) / C_0
    v = uvw[:, 1:2] * (FREQ0 + DFREQ * np.arange(NUM_CHAN)) / C_0
    w = uvw[:, 2:3] * (FREQ0 + DFREQ * np.arange(NUM_CHAN)) / C_0
    ph = 2 * np.pi * (np.multiply.outer(lmn_all[sel, 0], u)
                      + np.multiply.outer(lmn_all[sel, 1], v)
                      + np.multiply.outer(lmn_all[sel, 2], w))
    direct = np.einsum("prc,rc->p", np.exp(1j * ph), ref_vis)
    got = ref_img.ravel()[sel] * (rows * NUM_CHAN)
    assert np.max(np.abs(got - direct)) < 1e-8 * np.max(np.abs(direct))
    return dict(uvw=uvw, ref_vis=ref_vis, ref_img=ref_img, fov=fov,
                cell=cell, model=model)


def _geometry(grid_size, fov, cell):
    import ska_sdp_func.grid_data as g

    theta = math.sin(cell) * grid_size
    w_step = g.determine_w_step(theta, fov, 0.0, 0.0)
    H = g.determine_max_w_tower_height(
        SUBGRID, theta, fov, w_step, 8, 16 * 1024, 8, 16 * 1024,
        image_size=2 * SUBGRID, subgrid_frac=2.0 / 3.0)
    return theta, w_step, H


CASES = [
    # (location, uvw type, vis type, image type, grid size)
    ("cpu", np.float64, np.complex128, np.complex128, None),
    ("cpu", np.float64, np.complex64, np.complex128, None),
    ("cpu", np.float32, np.complex64, np.complex128, None),
    ("gpu", np.float64, np.complex128, np.complex128, None),
    ("gpu", np.float64, np.complex64, np.complex128, None),
    ("gpu", np.float32, np.complex64, np.complex128, None),
    ("gpu", np.float32, np.complex64, np.complex64, 1024),
]


@pytest.mark.parametrize("loc,uvw_t,vis_t,img_t,grid_size", CASES)
def test_run_and_check(device, reference, loc, uvw_t, vis_t, img_t,
                       grid_size):
    """run_and_check (test :408-558)."""
    import torch
    import ska_sdp_func.grid_data as g
    from ska_sdp_func.fourier_transforms import padded_fft_size

    if grid_size is None:
        grid_size = 2 * padded_fft_size(int(IMAGE_SIZE * 0.5), 1.2)
        assert grid_size == 616
    theta, w_step, H = _geometry(grid_size, reference["fov"],
                                 reference["cell"])
    uvw = reference["uvw"].astype(uvw_t)
    ref_vis = reference["ref_vis"]
    rows = len(uvw)
    img_padded = np.zeros((grid_size, grid_size), img_t)
    g.subgrid_add(img_padded, 0, 0, reference["model"].astype(img_t), 1.0)
    put = ((lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device))
           if loc == "gpu" else (lambda a: np.ascontiguousarray(a)))
    get = (lambda a: a.cpu().numpy()) if loc == "gpu" else (lambda a: a)
    common = (FREQ0, DFREQ, put(uvw), SUBGRID, theta, w_step, 0.0, 0.0, 8,
              16 * 1024, 8, 16 * 1024, 2.0 / 3.0, H, 0)
    vis = put(np.zeros((rows, NUM_CHAN), vis_t))
    g.wstack_wtower_degrid_all(put(img_padded), *common[:2], common[2],
                               *common[3:], vis)
    rms_vis = g.rms_diff(ref_vis, get(vis).astype(np.complex128))
    print(f"{loc} {np.dtype(uvw_t).name}/{np.dtype(vis_t).name}/"
          f"{np.dtype(img_t).name} G {grid_size}: rms vis {rms_vis:.3e}",
          end="")
    assert rms_vis < 1e-3
    img = put(np.zeros((grid_size, grid_size), img_t))
    g.wstack_wtower_grid_all(put(ref_vis.astype(vis_t)), *common[:2],
                             common[2], *common[3:], img)
    out = get(img).astype(np.complex128) / (rows * NUM_CHAN)
    trimmed = np.zeros((IMAGE_SIZE, IMAGE_SIZE), np.complex128)
    g.subgrid_cut_out(out, 0, 0, trimmed)
    rms_img = g.rms_diff(reference["ref_img"], trimmed)
    resid = np.zeros_like(trimmed)
    g.residual(reference["ref_img"], trimmed, resid)
    assert np.allclose(np.sqrt(np.mean(np.abs(resid) ** 2)), rms_img,
                       rtol=1e-6)
    print(f", rms image {rms_img:.3e}")
    assert rms_img < 1e-3


def test_fused_plane_image_kinds_agree(device, reference):
    """The fused image side of a complex-float plane (the sub-grid gather
    in the plane FFT's row pass, the corrected image update in its last
    column pass; es_fft_wstack.h) writes every image kind: the f32 image
    is Re of the c64 one, the c128 image the c64 one in double, all from
    the same c64 visibilities at grid 1024 (the c64 image is pinned to the
    reference recipe by test_run_and_check)."""
    import torch
    import ska_sdp_func.grid_data as g

    grid_size = 1024
    theta, w_step, H = _geometry(grid_size, reference["fov"],
                                 reference["cell"])
    put = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
    uvw = put(reference["uvw"].astype(np.float32))
    vis = put(reference["ref_vis"].astype(np.complex64))
    common = (FREQ0, DFREQ, uvw, SUBGRID, theta, w_step, 0.0, 0.0, 8,
              16 * 1024, 8, 16 * 1024, 2.0 / 3.0, H, 0)
    out = {}
    for t in (np.complex64, np.complex128, np.float32, np.float64):
        img = put(np.full((grid_size, grid_size), 0.25, t))  # overwritten
        g.wstack_wtower_grid_all(vis, *common[:2], common[2], *common[3:],
                                 img)
        out[t] = img.cpu().numpy().astype(np.complex128)
    ref = out[np.complex64]
    scale = np.max(np.abs(ref))
    assert np.max(np.abs(out[np.complex128] - ref)) <= 2e-6 * scale
    assert np.max(np.abs(out[np.float32] - ref.real)) <= 2e-6 * scale
    assert np.max(np.abs(out[np.float64] - ref.real)) <= 2e-6 * scale
    assert np.count_nonzero(out[np.float32].imag) == 0


def test_fused_plane_degrid_image_kinds_agree(device, reference):
    """Degridding through the fused image prologue (the degrid correction
    and checkerboard in the plane FFT's row pass, es_fft_wstack.h) reads
    every image kind: a real image gives the same visibilities as f32, f64,
    c64 or c128, from the reference model at grid 1024 (the c64 case is
    pinned to the reference recipe by test_run_and_check)."""
    import torch
    import ska_sdp_func.grid_data as g

    grid_size = 1024
    theta, w_step, H = _geometry(grid_size, reference["fov"],
                                 reference["cell"])
    put = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
    uvw = put(reference["uvw"].astype(np.float32))
    rows = len(reference["uvw"])
    common = (FREQ0, DFREQ, uvw, SUBGRID, theta, w_step, 0.0, 0.0, 8,
              16 * 1024, 8, 16 * 1024, 2.0 / 3.0, H, 0)
    out = {}
    for t in (np.complex64, np.complex128, np.float32, np.float64):
        img = np.zeros((grid_size, grid_size), t)
        g.subgrid_add(img, 0, 0, reference["model"].astype(t), 1.0)
        vis = put(np.zeros((rows, NUM_CHAN), np.complex64))
        g.wstack_wtower_degrid_all(put(img), *common[:2], common[2],
                                   *common[3:], vis)
        out[t] = vis.cpu().numpy().astype(np.complex128)
    ref = out[np.complex64]
    scale = np.max(np.abs(ref))
    assert scale > 0
    for t in (np.complex128, np.float32, np.float64):
        assert np.max(np.abs(out[t] - ref)) <= 2e-6 * scale, t
