"""Probe: does wstack_wtower_grid_all give the same image twice?"""
import sys
sys.path[:0] = ["ska-sdp-func_amd", "."]
import numpy as np
import torch
import ska_sdp_func.grid_data as g


def case(n_img, sub, rows, nchan, theta, fov, H, wplanes, seed=2):
    f0, df = 299792458.0, 299792458.0 / 200
    w_step = g.determine_w_step(theta, fov, 0.0, 0.0)
    rng = np.random.default_rng(seed)
    r = 0.4 * n_img / theta / 1.005 * np.sqrt(rng.random(rows))
    ph = 2 * np.pi * rng.random(rows)
    wmax = wplanes * H * w_step
    uvw = np.stack([r * np.cos(ph), r * np.sin(ph), rng.uniform(-wmax, wmax, rows)], 1)
    vis = rng.standard_normal((rows, nchan)) + 0j
    return f0, df, w_step, uvw, vis


def run(n_img, sub, rows, nchan, theta, fov, H, wplanes, vt, it, ut, frac=2 / 3):
    f0, df, w_step, uvw, vis = case(n_img, sub, rows, nchan, theta, fov, H, wplanes)
    d_uvw = torch.as_tensor(uvw.astype(ut), device="cuda")
    d_vis = torch.as_tensor(vis.astype(vt), device="cuda")
    outs = []
    for rep in range(3):
        img = torch.zeros((n_img, n_img), dtype=it, device="cuda")
        g.wstack_wtower_grid_all(d_vis, f0, df, d_uvw, sub, theta, w_step, 0.0, 0.0,
                                 8, 16384, 8, 16384, frac, H, 0, img)
        torch.cuda.synchronize()
        outs.append(img.cpu().numpy())
    s = np.abs(outs[0]).max()
    e1 = np.abs(outs[1] - outs[0]).max() / s
    e2 = np.abs(outs[2] - outs[0]).max() / s
    print(f"N {n_img} S {sub} R {rows} C {nchan} th {theta} H {H} wp {wplanes} "
          f"vis {np.dtype(vt).name} img {it} uvw {np.dtype(ut).name}: "
          f"repeat {e1:.2e} {e2:.2e}", flush=True)


c128, c64 = np.complex128, np.complex64
f64, f32 = torch.float64, torch.float32
run(512, 128, 20000, 2, 0.02, 0.016, 4.0, 3, c128, f64, np.float64)
run(512, 128, 20000, 2, 0.02, 0.016, 4.0, 3, c128, torch.complex128, np.float64)
run(512, 128, 20000, 2, 0.01, 0.008, 4.0, 3, c128, torch.complex128, np.float64)
run(1024, 128, 20000, 2, 0.02, 0.016, 4.0, 3, c128, torch.complex128, np.float64)
run(1024, 128, 100000, 2, 0.01, 0.008, 8.0, 5, c128, torch.complex128, np.float64)
run(512, 128, 2000, 1, 0.02, 0.016, 4.0, 3, c128, torch.complex128, np.float64)
run(512, 128, 20000, 2, 0.02, 0.016, 4.0, 0, c128, torch.complex128, np.float64)
run(512, 128, 20000, 2, 0.02, 0.016, 4.0, 3, c64, torch.complex64, np.float32)
run(512, 64, 20000, 2, 0.02, 0.016, 4.0, 3, c128, torch.complex128, np.float64)
run(512, 256, 20000, 2, 0.02, 0.016, 4.0, 3, c128, torch.complex128, np.float64)
