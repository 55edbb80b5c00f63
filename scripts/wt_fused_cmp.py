"""Fused (k_tower_dft) vs layer-by-layer w-tower gridding on one config-4
shaped case: run once per mode (SDP_WT_FUSED=1 / 0 in the environment,
read once per process), then compare.

  python scripts/wt_fused_cmp.py run OUT.npy [--rows R --image N ...]
  python scripts/wt_fused_cmp.py cmp A.npy B.npy
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func_amd"))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    if sys.argv[1] == "cmpvis":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        err = np.abs(a - b).max() / np.abs(b).max()
        rms = np.sqrt(np.mean(np.abs(a - b) ** 2) / np.mean(np.abs(b) ** 2))
        print(f"vis: max rel err {err:.3e}, rms rel err {rms:.3e}, "
              f"nonzero {np.count_nonzero(a)} / {np.count_nonzero(b)}")
        return
    if sys.argv[1] == "cmp":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        bd = a.shape[0] // 8
        ai, bi = a[bd:-bd, bd:-bd], b[bd:-bd, bd:-bd]
        err = np.abs(ai - bi).max() / np.abs(bi).max()
        rms = np.sqrt(np.mean(np.abs(ai - bi) ** 2) / np.mean(np.abs(bi) ** 2))
        print(f"max rel err {err:.3e}, rms rel err {rms:.3e}")
        print("norms", np.linalg.norm(ai), np.linalg.norm(bi))
        for name, x in (("T", a.T), ("flipud", a[::-1]), ("fliplr", a[:, ::-1]),
                        ("rot180", a[::-1, ::-1]), ("neg", -a)):
            xi = x[bd:-bd, bd:-bd]
            print(name, np.abs(xi - bi).max() / np.abs(bi).max())
        assert err < 1e-5, err
        return
    import torch
    import bench_wtower as bw
    ap = argparse.ArgumentParser()
    ap.add_argument("mode")
    ap.add_argument("out")
    ap.add_argument("--rows", type=int, default=300_000)
    ap.add_argument("--image", type=int, default=4096)
    ap.add_argument("--subgrid", type=int, default=256)
    ap.add_argument("--planes", type=int, default=4)
    ap.add_argument("--theta", type=float, default=0.04)
    ap.add_argument("--chan", type=int, default=1)
    ap.add_argument("--verbosity", type=int, default=0)
    ap.add_argument("--degrid", action="store_true")
    ap.add_argument("--f64", action="store_true")
    args = ap.parse_args()
    import ska_sdp_func.grid_data as g
    dev = torch.device("cuda:0")
    theta, fov, w_step, H = bw.geometry(args)
    uvw, vis = bw.make_inputs(torch, dev, args, H * w_step, 7)
    if args.f64:
        uvw = uvw.double()
        vis = vis.to(torch.complex128)
    N, S = args.image, args.subgrid
    image = torch.zeros((N, N), dtype=torch.float64 if args.f64 else
                        torch.float32, device=dev)
    if args.degrid:
        gen = torch.Generator(device=dev)
        gen.manual_seed(11)
        image = torch.randn((N, N), generator=gen, device=dev)
        if args.f64:
            image = image.double()
        b = N // 4
        image[:b] = 0
        image[-b:] = 0
        image[:, :b] = 0
        image[:, -b:] = 0
    common = (bw.C_0, bw.C_0 / 200, uvw, S, theta, w_step, 0.0, 0.0,
              bw.KW["support"], bw.KW["oversampling"], bw.KW["w_support"],
              bw.KW["w_oversampling"], 0.0, H)
    if args.degrid:
        out = torch.zeros_like(vis)
        g.wstack_wtower_degrid_all(image, *common, args.verbosity, out)
        torch.cuda.synchronize()
        out.zero_()
        t0 = time.perf_counter()
        g.wstack_wtower_degrid_all(image, *common, 1, out)
        torch.cuda.synchronize()
        print(f"{os.environ.get('SDP_WT_FUSED', '1')}: "
              f"{time.perf_counter() - t0:.3f} s")
        np.save(args.out, out.cpu().numpy())
        return
    g.wstack_wtower_grid_all(vis, *common, args.verbosity, image)
    torch.cuda.synchronize()
    image.zero_()
    t0 = time.perf_counter()
    g.wstack_wtower_grid_all(vis, *common, 1, image)
    torch.cuda.synchronize()
    print(f"{os.environ.get('SDP_WT_FUSED', '1')}: {time.perf_counter() - t0:.3f} s")
    np.save(args.out, image.cpu().numpy())


if __name__ == "__main__":
    main()
