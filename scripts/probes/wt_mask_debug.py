"""Probe: w-stack plane sets vs grid_all (INTEGRATION.md block 1 shape)."""
import sys
sys.path[:0] = ["ska-sdp-func_amd", "."]
import numpy as np
import torch
import ska_sdp_func.grid_data as g
from ska_sdp_func.grid_data.distributed import assign_planes, wstack_plane_loads

n_img, sub, rows, nchan = 512, 128, 20000, 2
theta, fov, H = 0.02, 0.016, 4.0
f0, df = 299792458.0, 299792458.0 / 200
w_step = g.determine_w_step(theta, fov, 0.0, 0.0)
rng = np.random.default_rng(2)
r = 0.4 * n_img / theta / 1.005 * np.sqrt(rng.random(rows))
ph = 2 * np.pi * rng.random(rows)
wmax = 3 * H * w_step
uvw_np = np.stack([r * np.cos(ph), r * np.sin(ph), rng.uniform(-wmax, wmax, rows)], 1)
uvw = torch.as_tensor(uvw_np, device="cuda")
vis = torch.as_tensor(rng.standard_normal((rows, nchan)) + 0j, device="cuda")
for frac in (0.0, 2 / 3):
    args = (f0, df, uvw, sub, theta, w_step, 0.0, 0.0, 8, 16384, 8, 16384, frac, H, 0)
    image = torch.zeros((n_img, n_img), dtype=torch.float64, device="cuda")
    g.wstack_wtower_grid_all(vis, *args, image)
    image2 = torch.zeros_like(image)
    g.wstack_wtower_grid_all(vis, *args, image2)
    torch.cuda.synchronize()
    print("frac", frac, "repeat err", float((image2 - image).abs().max() / image.abs().max()))
    for world in (1, 2, 3):
        tot = torch.zeros_like(image)
        for k in range(world):
            part = torch.zeros_like(image)
            g.wstack_wtower_grid_planes(vis, *args, part, k, world)
            tot += part
        torch.cuda.synchronize()
        print("  planes stride", world, float((tot - image).abs().max() / image.abs().max()))
    first, loads = wstack_plane_loads(uvw_np, f0, df, nchan, w_step, H)
    print("  first", first, "loads", loads.tolist())
    for world in (1, 2, 3):
        masks, cost = assign_planes(loads, world, fixed_cost=0.4 * loads.mean())
        tot = torch.zeros_like(image)
        for k in range(world):
            part = torch.zeros_like(image)
            g.wstack_wtower_grid_plane_set(vis, *args, part, first, torch.from_numpy(masks[k]))
            tot += part
        torch.cuda.synchronize()
        print("  mask world", world, masks.tolist(), float((tot - image).abs().max() / image.abs().max()))
