"""Synthetic visibility generators shared by the ES gridder tests."""
import numpy as np

C_LIGHT = 299792458.0


def disk_uvw(rng, num_rows, freq_max, pixel_size, frac=0.45, w_range=500.0):
    """(u, v) uniform in a disk sized so |u f/c * G * dx| <= frac * G.

    This keeps every visibility in-band.
    """
    umax = frac * C_LIGHT / (freq_max * pixel_size)
    r = umax * np.sqrt(rng.random(num_rows))
    th = 2.0 * np.pi * rng.random(num_rows)
    w = rng.uniform(-w_range, w_range, num_rows)
    return np.stack([r * np.cos(th), r * np.sin(th), w], axis=1)


def make_case(seed, num_rows, num_chan, image_size, fov_deg=2.0, f0=1e9,
              df=None, dbl=False, w_range=500.0, frac=0.45, weights="random"):
    rng = np.random.default_rng(seed)
    pixel_size = fov_deg * np.pi / 180.0 / image_size
    df = f0 / (2 * max(num_chan, 1)) if df is None else df
    freq = f0 + np.arange(num_chan) * df
    uvw = disk_uvw(rng, num_rows, freq[-1], pixel_size, frac, w_range)
    vis = (rng.standard_normal((num_rows, num_chan))
           + 1j * rng.standard_normal((num_rows, num_chan)))
    if weights == "random":
        wt = rng.uniform(0.5, 1.5, (num_rows, num_chan))
    else:
        wt = np.ones((num_rows, num_chan))
    if dbl:
        return (uvw, freq, vis.astype(np.complex128), wt, pixel_size)
    return (uvw.astype(np.float32), freq.astype(np.float32),
            vis.astype(np.complex64), wt.astype(np.float32), pixel_size)


def reference_test_case(do_single, num_vis=1000, num_chan=10, nxydirty=1024,
                        fov=2.0):
    """Data of the reference adjointness test
    (tests/grid_data/test_gridder_uvw_es_fft.py:532-560 of ska-sdp-func)."""
    np.random.seed(40)
    pixel_size_rad = fov * np.pi / 180 / nxydirty
    f_0 = 1e9
    freqs = f_0 + np.arange(num_chan) * (f_0 / num_chan)
    uvw = (np.random.rand(num_vis, 3) - 0.5) / (pixel_size_rad * f_0 / C_LIGHT)
    test_vis = (np.random.rand(num_vis, num_chan) - 0.5
                + 1j * (np.random.rand(num_vis, num_chan) - 0.5))
    test_dirty_image = np.random.rand(nxydirty, nxydirty) - 0.5
    weight = np.ones([num_vis, num_chan])
    if do_single:
        test_vis = test_vis.astype(np.complex64)
        test_dirty_image = test_dirty_image.astype(np.float32)
        freqs = freqs.astype(np.float32)
        uvw = uvw.astype(np.float32)
        weight = weight.astype(np.float32)
    return uvw, freqs, test_vis, weight, test_dirty_image, pixel_size_rad


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.complex128)
    b = np.asarray(b, dtype=np.complex128)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))
