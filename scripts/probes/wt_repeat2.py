"""Probe: repeatability of the c128 w-stack gridder, test data vs probe data."""
import sys
sys.path[:0] = ["ska-sdp-func_amd", ".", "tests"]
import numpy as np
import torch
import ska_sdp_func.grid_data as g
import wtower_data as wd


def reps(tag, uvw, vis, N, S, theta, w_step, H, f0, df, n=3):
    d_uvw = torch.as_tensor(uvw, device="cuda")
    d_vis = torch.as_tensor(vis, device="cuda")
    outs = []
    for _ in range(n):
        img = torch.zeros((N, N), dtype=torch.complex128, device="cuda")
        g.wstack_wtower_grid_all(d_vis, f0, df, d_uvw, S, theta, w_step, 0.0,
                                 0.0, 8, 16384, 8, 16384, 0.0, H, 0, img)
        torch.cuda.synchronize()
        outs.append(img.cpu().numpy())
    s = np.abs(outs[0]).max()
    print(tag, "max", s, "finite", [bool(np.isfinite(o).all()) for o in outs],
          "repeat", [float(np.abs(o - outs[0]).max() / s) for o in outs[1:]],
          flush=True)
    return outs[0]


N, S, R, C = 1024, 128, 100000, 2
c = wd.wstack_case(num_rows=R, num_chan=C, image_size=N, seed=4,
                   w_tower_height=8.0, w_planes=5.0)
rng = np.random.default_rng(5)
y = rng.normal(size=(R, C)) + 1j * rng.normal(size=(R, C))
args = (N, S, c["theta"], c["w_step"], c["H"], c["f0"], c["df"])
reps("test data, complex vis", c["uvw"], y, *args)
reps("test data, real vis", c["uvw"], y.real + 0j, *args)
reps("test data, complex vis again", c["uvw"], y, *args)
y2 = y.copy()
y2[:, 1] = 0
reps("test data, chan 1 zero", c["uvw"], y2, *args)
reps("test data, imag*1e-3", c["uvw"], y.real + 1e-3j * y.imag, *args)
