#!/usr/bin/env python3
"""Benchmark of the w-stacking x w-towers imaging driver at SURVEY.md
section 8(d) config 4: 10M rows x 1 channel, image 16384^2, sub-grid 256,
W = W_w = 8, oversampling 16384, subgrid_frac 2/3, w_tower_height from
determine_max_w_tower_height, w spread over 32 w-stack planes.

A "step" is one wstack_wtower_grid_all over all rows. With --gpus N (one
process per GPU, torchrun), the w-stack planes are sharded across the ranks
(grid_plane_set with the planes assigned by a cost model: visibilities per
plane + a fixed image-side cost, heaviest plane to the least-loaded rank;
ska_sdp_func.grid_data.distributed.assign_planes) and the rank
images are summed on rank 0 with one RCCL reduce inside the timed region;
total work is fixed ("scaling": "strong"). Inputs are generated in HBM
(uvw f32, vis c64, f0 = c so that metres are wavelengths).

Prints one JSON line (same field layout as bench.py).

  python bench_wtower.py [--rows 10000000 --image 16384 --steps 3]
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func_amd"))
sys.path.insert(0, ROOT)

C_0 = 299792458.0
F32_PEAK_TFLOPS = 157.3
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E (MI355X_MICROARCH.md)
KW = dict(support=8, oversampling=16384, w_support=8, w_oversampling=16384)
# Image-side cost of one w-stack plane (plane FFT, cut-out / update, grid
# gather) in units of the mean plane's visibility load: ~8 ms against
# ~20 ms of towers per plane at config 4 (profiles/r4_wtower_kernel_stats).
PLANE_FIXED = 0.4


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--chan", type=int, default=1)
    ap.add_argument("--image", type=int, default=16384)
    ap.add_argument("--subgrid", type=int, default=256)
    ap.add_argument("--planes", type=int, default=32)
    ap.add_argument("--theta", type=float, default=0.04)
    ap.add_argument("--degrid", action="store_true")
    ap.add_argument("--verbosity", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-task-stride", type=int, default=8)
    return ap.parse_args()


def geometry(args):
    """theta, fov, w_step, w_tower_height (the reference's C test recipe,
    test_gridder_wtower_uvw.cpp:437-452)."""
    import ska_sdp_func.grid_data as g
    theta = args.theta
    fov = 0.8 * theta
    w_step = g.determine_w_step(theta, fov, 0.0, 0.0)
    H = g.determine_max_w_tower_height(
        args.subgrid, theta, fov, w_step, KW["support"], KW["oversampling"],
        KW["w_support"], KW["w_oversampling"], image_size=2 * args.subgrid,
        subgrid_frac=2.0 / 3.0)
    return theta, fov, w_step, float(H)


def make_inputs(torch, dev, args, w_stack_dist, seed):
    """(u, v) uniform in a disk reaching 0.45 of the grid half-width at the
    top channel; w uniform over exactly args.planes w-stack planes."""
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    R = args.rows
    f_max = 1.0 + (args.chan - 1) / 200.0
    r_max = 0.45 * args.image / args.theta / f_max
    r = r_max * torch.sqrt(torch.rand(R, generator=gen, device=dev,
                                      dtype=torch.float64))
    ph = 2 * math.pi * torch.rand(R, generator=gen, device=dev,
                                  dtype=torch.float64)
    half = args.planes / 2
    w = (torch.rand(R, generator=gen, device=dev, dtype=torch.float64)
         * args.planes - half - 0.5) * w_stack_dist
    uvw = torch.stack([r * torch.cos(ph), r * torch.sin(ph), w], dim=1)
    uvw = uvw.to(torch.float32).contiguous()
    vis = torch.complex(
        torch.randn((R, args.chan), generator=gen, device=dev),
        torch.randn((R, args.chan), generator=gen, device=dev)).contiguous()
    return uvw, vis


def cpu_baseline(uvw_dev, vis_dev, args, theta, w_step, H):
    """C/OpenMP port of the reference CPU grid_all (oracle/wtower_port.c,
    checked against the numpy restatement by tests/test_wtower_port.py) on
    a bounded sample of the same inputs, on the job's host-CPU share.

    Sample: the central w-stack plane. Its sub-grid towers are run for
    every k-th non-empty sub-grid task (k = --cpu-task-stride; each task is
    one sub-grid tower, the reference's unit of CPU parallelism), then the
    whole plane's FFT, grid correction and accumulation. The plane time is
    projected as t_towers * (tasks present / tasks run) + t_plane, and the
    value is the plane's visibilities over that time. The per-call set-up
    (kernel tables, PSWF tables, bounds) is not timed.
    """
    import numpy as np
    from bench import host_cpus
    from oracle import wtower_port as wp
    cpus = host_cpus()
    threads = wp.set_threads(cpus["usable"])
    uvw = uvw_dev.cpu().numpy().astype(np.float64)
    vis = vis_dev.cpu().numpy()
    plan = wp.Plan(vis, C_0, C_0 / 200, uvw, args.image, args.subgrid, theta,
                   w_step, KW["support"], KW["oversampling"],
                   KW["w_support"], KW["w_oversampling"], 0.0, H)
    planes = plan.planes()
    iw = planes[len(planes) // 2]
    k = max(1, args.cpu_task_stride)
    t0 = time.perf_counter()
    n_s, done, present = plan.grid_towers(iw, k, 0)
    t1 = time.perf_counter()
    image = np.zeros((args.image, args.image), np.float32)
    plan.finish_plane(iw, image)
    t2 = time.perf_counter()
    # all visibilities of the plane (the stride-1 clamp count, no gridding)
    n_plane = int(np.sum(_plane_vis(uvw, args.chan, H * w_step, iw)))
    t_proj = (t1 - t0) * present / max(done, 1) + (t2 - t1)
    return {"value": round(n_plane / t_proj / 1e6, 6), "unit": "Mvis/s",
            "cores": threads, "kind": "port", "host_cpus": cpus,
            "sample": (f"oracle/wtower_port.c (C/OpenMP, {threads} threads) "
                       f"w-stack plane {iw} of {len(planes)}: towers of "
                       f"{done} of {present} non-empty sub-grid tasks "
                       f"({n_s} vis, {t1 - t0:.1f} s), then the full "
                       f"{args.image}^2 plane FFT + correction + "
                       f"accumulation ({t2 - t1:.1f} s); projected plane "
                       f"time {t_proj:.1f} s for {n_plane} vis"),
            "towers_s": round(t1 - t0, 3), "plane_fft_correct_s":
            round(t2 - t1, 3)}


def _plane_vis(uvw, num_chan, ws_dist, iw):
    """Visibilities of each row on w-stack plane iw (clamp_channels)."""
    from oracle import wtower_oracle as wo
    import numpy as np
    R = uvw.shape[0]
    s, e = wo.clamp_rows_vec(uvw[:, 2], C_0, C_0 / 200,
                             np.zeros(R, np.int64),
                             np.full(R, num_chan, np.int64),
                             iw * ws_dist - ws_dist / 2,
                             (iw + 1) * ws_dist - ws_dist / 2)
    return e - s


def roofline(tm, kernel):
    """Roofline object of a fused tower kernel from the library's event
    timing. Algorithmic flops (w-towers): every
    visibility updates all S^2 pixels of its sub-grid image by a complex
    rank-1 term (8 flops per pixel) and every sub-grid w-layer steps the
    S^2-pixel Horner recurrence (one complex multiply-add, 8 flops per
    pixel); bound: f32 matrix/vector peak (both 157.3 TFLOP/s on MI355X)."""
    if not tm or not tm["launches"] or tm["kernel_ms"] <= 0:
        return None
    s2 = tm["subgrid_size"] ** 2
    flops = 8.0 * s2 * (tm["vis"] + tm["layers"]) / tm["launches"]
    avg_s = tm["kernel_ms"] * 1e-3 / tm["launches"]
    achieved = flops / avg_s / 1e12
    return {"kernel": kernel, "bound": "mfma",
            "achieved": round(achieved, 2), "peak": F32_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / F32_PEAK_TFLOPS, 4),
            "traffic": None, "avg_launch_ms": round(1e3 * avg_s, 3),
            "launches": tm["launches"],
            "algorithmic_flops_per_launch": flops}


def image_side(ms_per_call, tm, n_planes, G):
    """Roofline of the image side of a call (everything but the tower
    kernels: binning, sub-grid FFTs, gather / cut-out, plane FFT, image
    update): its time is the call's minus the live-timed tower kernels',
    per w-stack plane; its bytes per plane are SURVEY 8(d)'s 7 G^2 s_g
    (zero + sub-grid adds + one FFT read/write + grid-correct RMW + image
    accumulate, complex-float grid). HBM bound."""
    if not tm or not tm["launches"] or n_planes <= 0:
        return None
    t_plane = (ms_per_call - tm["kernel_ms"]) / n_planes
    if t_plane <= 0:
        return None
    algo = 7.0 * G * G * 8
    achieved = algo / (t_plane * 1e-3) / 1e9
    return {"what": "non-tower time per w-stack plane (call minus the "
                    "event-timed tower kernels)",
            "bound": "hbm", "ms_per_plane": round(t_plane, 3),
            "algorithmic_bytes_per_plane": algo,
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
            "planes": n_planes}


def main():
    args = parse()
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    import ska_sdp_func.grid_data as g

    theta, fov, w_step, H = geometry(args)
    uvw, vis = make_inputs(torch, dev, args, H * w_step, 20251015 + 4)
    N, S = args.image, args.subgrid
    image = torch.zeros((N, N), dtype=torch.float32, device=dev)
    common = (C_0, C_0 / 200, uvw, S, theta, w_step, 0.0, 0.0,
              KW["support"], KW["oversampling"], KW["w_support"],
              KW["w_oversampling"], 0.0, H)

    # Multi-GPU: the w-stack planes are dealt to the ranks by a cost model
    # (visibilities per plane + a fixed image-side cost per plane, longest
    # first to the least-loaded rank), outside the timed region.
    from ska_sdp_func.grid_data.distributed import (assign_planes,
                                                    plane_balance,
                                                    wstack_plane_loads)
    first, loads = wstack_plane_loads(uvw, C_0, C_0 / 200, args.chan, w_step,
                                      H)
    masks, pcost = assign_planes(loads, world,
                                 fixed_cost=PLANE_FIXED * loads.mean())
    my_mask = torch.from_numpy(masks[rank]).to(dev)

    def grid_step(verbosity=0):
        g.wstack_wtower_grid_plane_set(vis, *common, verbosity, image, first,
                                       my_mask)
        if dist is not None:
            dist.reduce(image, dst=0)

    def barrier():
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        grid_step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        grid_step()
    barrier()
    t_grid = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([t_grid], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_grid = float(t.item())
    total_vis = args.rows * args.chan
    value = total_vis * args.steps / t_grid / 1e6

    # Roofline of the dominant kernel (k_tower_dft), timed by HIP events
    # around each launch inside the library, in a separate step so that the
    # event synchronisation stays out of the timed loop.
    g.wstack_wtower_enable_timing(True)
    grid_step()
    barrier()
    tm_grid = g.wstack_wtower_get_timing()
    roof = roofline(tm_grid, "k_tower_dft")
    g.wstack_wtower_enable_timing(False)
    # Occupied w-stack planes of this rank (one tower launch each unless a
    # plane's sub-grids need several groups).
    n_planes = int(((np.asarray(loads) > 0) & np.asarray(masks[rank])).sum())
    img_side = image_side(1e3 * t_grid / args.steps, tm_grid, n_planes, N)
    if args.verbosity:
        grid_step(args.verbosity)
        barrier()

    degrid = None
    if args.degrid:
        out = torch.zeros_like(vis)
        for _ in range(args.warmup):
            g.wstack_wtower_degrid_plane_set(image, *common, 0, out, first,
                                             my_mask)
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            g.wstack_wtower_degrid_plane_set(image, *common, 0, out, first,
                                             my_mask)
        barrier()
        t_deg = time.perf_counter() - t0
        g.wstack_wtower_enable_timing(True)
        g.wstack_wtower_degrid_plane_set(image, *common, 0, out, first,
                                         my_mask)
        barrier()
        tm_deg = g.wstack_wtower_get_timing()
        droof = roofline(tm_deg, "k_tower_idft")
        g.wstack_wtower_enable_timing(False)
        degrid = {"mvis_s": round(total_vis * args.steps / t_deg / 1e6, 3),
                  "ms_per_step": round(1e3 * t_deg / args.steps, 2),
                  "roofline": droof,
                  "image_side": image_side(1e3 * t_deg / args.steps, tm_deg,
                                           n_planes, N)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(uvw, vis, args, theta, w_step, H)
        except Exception as exc:  # baseline failure must not hide the bench
            cpu = {"value": None, "unit": "Mvis/s", "cores": None,
                   "kind": "port", "sample": f"failed: {exc!r}"}

    if rank == 0:
        line = {
            "metric": "Mvis/s gridded",
            "value": round(value, 3),
            "unit": "Mvis/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * t_grid / args.steps, 2),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (config-4 distribution, generated in HBM)",
            "config": {
                "workload": (f"wstack_wtower_grid_all, {args.rows} rows x "
                             f"{args.chan} chan, image {N}^2, sub-grid {S},"
                             f" W = W_w = 8, os 16384, {args.planes} w-stack "
                             f"planes (sharded over {world} GPU(s))"),
                "theta": theta, "fov": fov, "w_step": w_step,
                "w_tower_height": H,
                "parallelism": f"w-stack planes / {world}",
                "plane_balance": round(plane_balance(pcost), 4),
            },
            "roofline": roof,
            "image_side": img_side,
            "degrid": degrid,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
