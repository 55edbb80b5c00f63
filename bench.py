#!/usr/bin/env python3
"""Benchmark: Mvis/s gridded by the MI355X-native ES-FFT gridder.

Workload (BASELINE.json configs[1]):
  10M synthetic visibility rows x 1 channel, image 5440^2, epsilon 1e-5,
  f32 -> uv grid 8192^2, support 8; 2-D (no w-stacking); uvw uniform in a
  disk keeping every visibility in-band; complex-normal vis; unit weights.
  Inputs are generated directly in HBM (seed 20251015 + 2 + rank).

A step = one full sdp_grid_uvw_es_fft call through the C ABI (bucketing,
MFMA tile scatter, pruned fused inverse FFT 8192^2 with the screen and grid
correction in its last pass).
value = visibilities gridded per second over the whole job (all ranks).
The degridding half of the config-2 round trip is timed afterwards with the
same step count and reported in "degrid"; "roundtrip_mvis_s" = R / (t_grid +
t_degrid).

Multi-GPU (torchrun, one process per GPU, RCCL): weak scaling -- every rank
grids its own 10M rows (a row shard of the job) into a partial image, then
the partial images are summed onto rank 0 with one RCCL reduce (default,
--reduce image: 5440^2 f32 = 118 MB); step k's reduce runs on RCCL's stream
while step k + 1 grids into a second image buffer (every reduce completes
before the clock stops; --no-overlap serialises them). The north star's
other form -- the per-GPU 8192^2 grids (512 MiB) reduced before a single
FFT on rank 0 -- is timed after it and reported in "grid_reduce_mode".

"config3": BASELINE config 3 at every N -- 10M rows x 64 channels IN TOTAL
(1.0-1.49 GHz), rows sharded over the ranks, per-rank scatter into a
private grid, one RCCL reduce of the grids, one FFT + screen + correction on
rank 0 (strong scaling); the reduce is also timed alone ("reduce_ms").

Roofline: the dominant hand-written kernel's algorithmic bytes per launch
divided by its HIP-event duration (library timing on the launch stream).
"""
import argparse
import csv
import glob
import json
import os
import re
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func_amd"))
sys.path.insert(0, ROOT)

C_LIGHT = 299792458.0
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3        # MI355X_MICROARCH.md: FP32 vector = f32 MFMA


def csrc_sha16(root=ROOT):
    """sha256 (16 hex digits) of the native sources the library is built
    from: ska-sdp-func_amd/csrc/**, include/** and the Makefile (paths and
    contents, sorted). profiles/pmc_traffic.json records the value of the
    build its counters were taken on; bench.py reports that traffic only
    when the current sources hash to the same value."""
    import hashlib
    h = hashlib.sha256()
    files = []
    for sub in ("ska-sdp-func_amd/csrc", "include"):
        for dp, _, fns in os.walk(os.path.join(root, sub)):
            files += [os.path.join(dp, f) for f in fns]
    files.append(os.path.join(root, "ska-sdp-func_amd", "Makefile"))
    for f in sorted(files):
        if "__pycache__" in f or not os.path.isfile(f):
            continue
        h.update(os.path.relpath(f, root).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--chan", type=int, default=1)
    ap.add_argument("--image", type=int, default=5440)
    ap.add_argument("--eps", type=float, default=1e-5)
    ap.add_argument("--reduce", choices=["image", "grid"], default="image")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-rows", type=int, default=10_000_000)
    ap.add_argument("--no-degrid", action="store_true")
    ap.add_argument("--no-config3", action="store_true",
                    help="skip the config-3 measurement (10M rows x 64 "
                         "channels in total, sharded, RCCL grid reduce)")
    ap.add_argument("--c3-rows", type=int, default=10_000_000)
    ap.add_argument("--c3-chan", type=int, default=64)
    ap.add_argument("--c3-steps", type=int, default=3)
    ap.add_argument("--no-wstack", action="store_true",
                    help="skip the 3-D (w-stacking) line at the config-2 "
                         "workload")
    ap.add_argument("--no-overlap", action="store_true",
                    help="multi-GPU: wait for each step's reduce before the "
                         "next step (default: reduce of step k overlaps "
                         "step k + 1)")
    return ap.parse_args()


def make_inputs(torch, dev, rows, chan, image, seed):
    """Synthetic config-2 data generated on the device."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    fov_deg = 2.0
    px = fov_deg * np.pi / 180.0 / image
    f0 = 1e9
    df = 0.5 * f0 / max(chan, 1)
    freq = torch.tensor(f0 + np.arange(chan) * df, dtype=torch.float32,
                        device=dev)
    fmax = float(f0 + (chan - 1) * df)
    umax = 0.45 * C_LIGHT / (fmax * px)
    r = umax * torch.sqrt(torch.rand(rows, generator=g, device=dev))
    th = 2.0 * np.pi * torch.rand(rows, generator=g, device=dev)
    w = (torch.rand(rows, generator=g, device=dev) - 0.5) * 1000.0
    uvw = torch.stack([r * torch.cos(th), r * torch.sin(th), w], 1).float()
    vis = torch.complex(torch.randn(rows, chan, generator=g, device=dev),
                        torch.randn(rows, chan, generator=g, device=dev))
    weight = torch.ones(rows, chan, dtype=torch.float32, device=dev)
    return uvw.contiguous(), freq, vis.contiguous(), weight, px


def scatter_bytes(rows, chan, G):
    """Algorithmic HBM bytes of the gridding scatter:
    vis + weight read, uvw read, grid written once."""
    return rows * chan * (8 + 4) + rows * 3 * 4 + chan * 4 + G * G * 8


def es_flops_per_vis(W):
    """SURVEY 8(d) guard roofline: per visibility 2W ES evaluations (exp +
    sqrt, 2 flops each) + 5 W^2 for the separable tap products and the
    complex accumulation: 352 at W = 8 (the survey rounds to ~360), 96 at
    W = 4."""
    return 5 * W * W + 4 * W


def fp32_roofline(n_vis, W, ms):
    """FP32-vector guard: algorithmic flops of n_vis visibilities over ms
    against the 157.3 TFLOP/s FP32 peak (vector = f32 matrix rate)."""
    flops = n_vis * es_flops_per_vis(W)
    tfs = flops / (ms * 1e-3) / 1e12 if ms else None
    return {"bound": "fp32", "flops_per_vis": es_flops_per_vis(W),
            "flops_per_launch": flops,
            "achieved": round(tfs, 3) if tfs else None,
            "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tfs / FP32_PEAK_TFLOPS, 4) if tfs else None}


def fft_bytes(G):
    """One read + one write of the complex64 grid."""
    return 2 * G * G * 8


def gridding_bytes(rows, chan, G, n):
    """Whole gridding call: scatter + FFT + screen + corr."""
    return (scatter_bytes(rows, chan, G) + fft_bytes(G)
            + n * n * (8 + 4) + 2 * n * n * 4)


def host_cpus():
    """CPUs this process may use, and the machine's count.

    nproc / os.cpu_count() report every CPU of the host; a GPU box grants
    each job a share of them (its affinity mask and cgroup CPU quota), and
    running more threads than the share only time-slices them. The CPU
    baselines use the share and report all three figures.
    """
    total = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = total
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        quota = None
    usable = min(affinity, quota) if quota else affinity
    env = os.environ.get("OMP_NUM_THREADS")
    return {"nproc": total, "affinity": affinity, "cgroup_quota": quota,
            "omp_num_threads_env": int(env) if env and env.isdigit() else None,
            "usable": usable}


def h2d_time(torch, dev, tensors, reps=3):
    """Host -> device copy of a call's inputs (reported beside
    the Mvis/s, never part of it): the device tensors are staged once into
    pinned host buffers, then copied back to HBM reps times on the current
    stream (non-blocking, one synchronisation per rep). Returns the mean ms
    per copy of all tensors and the bytes moved."""
    host = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            for t in tensors]
    for h, t in zip(host, tensors):
        h.copy_(t)
    nbytes = sum(t.numel() * t.element_size() for t in tensors)
    torch.cuda.synchronize(dev)
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        for h, t in zip(host, tensors):
            t.copy_(h, non_blocking=True)
        torch.cuda.synchronize(dev)
        times.append(time.perf_counter() - t0)
    del host
    ms = 1e3 * sum(times) / len(times)
    return {"h2d_ms": round(ms, 3), "bytes": nbytes,
            "GBs": round(nbytes / (ms * 1e-3) / 1e9, 1),
            "what": "uvw + vis + weight from pinned host memory"}


def cpu_baseline(args, G, support, beta, uv_scale):
    """Oracle ('port') CPU gridder timed on the host cores.

    The whole config-2 gridding call on the CPU: the stripe-binned OpenMP
    f32 scatter of oracle/es_oracle.c (same taps as the reference), a
    multi-threaded pocketfft (scipy) inverse FFT of the grid, and the crop +
    checkerboard + correction of the image in numpy. Run on the same number
    of rows as the GPU step when --cpu-sample-rows >= --rows, else on that
    many rows with the scatter time scaled linearly (the FFT and image steps
    do not depend on the row count).
    """
    import scipy.fft

    from oracle import es_oracle

    host = host_cpus()
    threads = host["usable"]
    lib = es_oracle.lib()
    lib.oracle_set_threads(threads)
    n_s = min(args.cpu_sample_rows, args.rows)
    rng = np.random.default_rng(20251015 + 2)
    px = 2.0 * np.pi / 180.0 / args.image
    umax = 0.45 * C_LIGHT / (1e9 * px)
    r = umax * np.sqrt(rng.random(n_s))
    th = 2 * np.pi * rng.random(n_s)
    uvw = np.stack([r * np.cos(th), r * np.sin(th),
                    rng.uniform(-500, 500, n_s)], 1).astype(np.float32)
    del r, th
    vis = (rng.standard_normal((n_s, 1)) + 1j * rng.standard_normal(
        (n_s, 1))).astype(np.complex64)
    wt = np.ones((n_s, 1), np.float32)
    freq = np.array([1e9], np.float32)
    grid = np.zeros((G, G), np.complex64)
    t0 = time.perf_counter()
    used = lib.oracle_es_grid_f32_omp(n_s, 1, es_oracle._ptr(uvw),
                                      es_oracle._ptr(freq),
                                      es_oracle._ptr(vis), es_oracle._ptr(wt),
                                      G, support, float(np.float32(beta)),
                                      float(np.float32(uv_scale)),
                                      es_oracle._ptr(grid))
    t_scatter = time.perf_counter() - t0
    t0 = time.perf_counter()
    layer = scipy.fft.ifft2(grid, norm="forward", workers=threads,
                            overwrite_x=True)
    h, gc = args.image // 2, G // 2
    off = np.arange(-h, h)
    sgn = np.where(((off[:, None] + off[None, :]) & 1) != 0, -1.0, 1.0)
    img = (layer[gc - h:gc + h, gc - h:gc + h].real * sgn).astype(np.float32)
    img *= np.float32(1.0001)   # separable correction multiply
    t_fft_img = time.perf_counter() - t0
    del layer, img, grid
    scale = args.rows * args.chan / n_s
    t_job = t_scatter * scale + t_fft_img
    return {
        "value": args.rows * args.chan / t_job / 1e6,
        "unit": "Mvis/s",
        "cores": int(used),
        "host_cpus": host,
        "kind": "port",
        "sample": (f"oracle/es_oracle.c stripe-binned OpenMP f32 scatter of "
                   f"{n_s} config-2 rows ({t_scatter:.3f} s"
                   + (f", x{scale:.2f} to {args.rows} rows" if scale != 1
                      else "")
                   + f") + scipy pocketfft ifft2 {G}^2 c64 on {threads} "
                   f"threads + crop/checkerboard/correction "
                   f"({t_fft_img:.3f} s); {int(used)} threads = the CPUs "
                   f"this job may use (affinity {host['affinity']}, cgroup "
                   f"quota {host['cgroup_quota']}) of the host's "
                   f"{host['nproc']}"),
    }


def run_config3(args, torch, dev, dist, world, rank):
    """BASELINE config 3: 10M rows x 64 channels IN TOTAL, rows sharded
    over the ranks (strong scaling). Two ways to combine the ranks, both
    timed at N > 1:
      grid  -- the north star's form: each rank scatters its shard into a
               private uv grid, one RCCL reduce of the 8192^2 complex64
               grids (512 MiB) onto rank 0, one FFT + screen + correction
               there;
      image -- each rank runs the whole gridding call on its shard into a
               partial image, one RCCL reduce of the 5440^2 f32 images
               (118 MB) onto rank 0.
    The top-level mvis_s / ms_per_step are the faster mode's. With one GPU
    the whole call runs on it (no collective). Each reduce is also timed
    alone (reduce_ms)."""
    from ska_sdp_func.grid_data import GridderUvwEsFft
    from ska_sdp_func.grid_data.distributed import (grid_sharded,
                                                    predicted_speedup,
                                                    shard_rows)

    r0, r1 = shard_rows(args.c3_rows, rank, world)
    uvw, freq, vis, weight, px = make_inputs(
        torch, dev, r1 - r0, args.c3_chan, args.image,
        20251015 + 3 + rank)
    dirty = torch.zeros((args.image, args.image), dtype=torch.float32,
                        device=dev)
    plan = GridderUvwEsFft(uvw, freq, vis, weight, dirty, px, px, args.eps,
                           False)
    plan.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    G = plan.grid_size
    grid_buf = (torch.empty((G, G), dtype=torch.complex64, device=dev)
                if world > 1 else None)
    # Mode "grid" reduces the row spectra of the Hermitian part (fused f32
    # plans) instead of the whole grid: what travels per rank.
    spec = plan.row_spectra()
    grid_red_bytes = (spec[0] * spec[2] * 8 if spec else G * G * 8)

    def sync():
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(dev)

    def timed(step):
        step()
        sync()
        t0 = time.perf_counter()
        for _ in range(args.c3_steps):
            step()
        sync()
        t = time.perf_counter() - t0
        if dist is not None:
            tt = torch.tensor([t], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t = float(tt.item())
        return t

    def reduce_ms(buf):
        n_red = 3
        sync()
        t0 = time.perf_counter()
        for _ in range(n_red):
            dist.reduce(buf, dst=0)
        sync()
        return round(1e3 * (time.perf_counter() - t0) / n_red, 3)

    total = args.c3_rows * args.c3_chan
    modes = {}
    if world == 1:
        def step():
            dirty.zero_()
            plan.grid_uvw_es_fft(uvw, freq, vis, weight, dirty)
        t = timed(step)
        modes["single"] = {"mvis_s": round(total * args.c3_steps / t / 1e6,
                                           3),
                           "ms_per_step": round(1e3 * t / args.c3_steps, 3),
                           "reduce_ms": None}
    else:
        for mode in ("grid", "image"):
            def step(mode=mode):
                dirty.zero_()
                grid_sharded(plan, uvw, freq, vis, weight, dirty, dist,
                             mode=mode, dst=0, grid_buf=grid_buf)
            t = timed(step)
            modes[mode] = {
                "mvis_s": round(total * args.c3_steps / t / 1e6, 3),
                "ms_per_step": round(1e3 * t / args.c3_steps, 3),
                "reduce": (f"per-GPU row pass of the inverse FFT, then "
                           f"one RCCL reduce of the row spectra "
                           f"({grid_red_bytes / 1e6:.0f} MB; the whole "
                           f"{G}^2 grid is {G * G * 8 / 2**20:.0f} MiB) "
                           f"before the column passes on rank 0"
                           if mode == "grid" else
                           "RCCL reduce of the per-GPU partial images "
                           f"({args.image}^2 f32, "
                           f"{args.image ** 2 * 4 / 1e6:.0f} MB)"),
                "reduce_ms": reduce_ms(
                    torch.empty(grid_red_bytes // 8, dtype=torch.complex64,
                                device=dev) if mode == "grid" else dirty),
            }
    # Per-phase device times of one whole call on this rank's shard (HIP
    # events on the plan stream, summed over the call's row batches),
    # outside the timed loops: the roofline of the dominant kernel and the
    # inputs of the scaling model.
    plan.enable_timing(True)
    dirty.zero_()
    plan.grid_uvw_es_fft(uvw, freq, vis, weight, dirty)
    tm = plan.get_timing() or {}
    plan.enable_timing(False)
    sync()
    phases = {k: round(tm.get(k, 0.0), 4)
              for k in ("bucket", "tile_kernel", "fft", "image")}
    n_shard = (r1 - r0) * args.c3_chan
    t_tile = phases["tile_kernel"]
    sbytes = scatter_bytes(r1 - r0, args.c3_chan, G)
    hbm = (sbytes / (t_tile * 1e-3) / 1e9) if t_tile else None
    roofline = {
        "kernel": "k_scatter_tab (all row batches of the call)",
        "bound": "hbm",
        "achieved": round(hbm, 1) if hbm else None,
        "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(hbm / HBM_PEAK_GBS, 4) if hbm else None,
        "algorithmic_bytes_per_call": sbytes,
        "launch_ms": t_tile,
        "fp32": fp32_roofline(n_shard, plan.support, t_tile),
        "call_fp32_frac": fp32_roofline(n_shard, plan.support,
                                        sum(phases.values()))["frac"],
    }
    # Strong-scaling model from the one-GPU phases (at N > 1 with the
    # measured reduce times): the bucketing + tile kernels divide over the
    # ranks, the FFT + image steps do not.
    pred = None
    if world == 1:
        t_sc = phases["bucket"] + phases["tile_kernel"]
        t_fi = phases["fft"] + phases["image"]
        pred = {"n_gpus": 8,
                "modes": predicted_speedup(t_sc, t_fi, 8, grid_red_bytes,
                                           args.image ** 2 * 4,
                                           grid_packed=spec is not None),
                "grid_mode": ("per-rank row pass, reduce of the (G/2 + 1) x "
                              "M Hermitian row spectra, column passes on "
                              "the destination" if spec else
                              "reduce of the whole grid"),
                "inputs": {"scatter_ms": round(t_sc, 3),
                           "fft_image_ms": round(t_fi, 3)}}
    best = max(modes, key=lambda k: modes[k]["mvis_s"])
    h2d = h2d_time(torch, dev, [uvw, vis, weight])
    out = {
        "workload": (f"ES-FFT gridding, {args.c3_rows} rows x "
                     f"{args.c3_chan} chan in total (1.0-1.49 GHz), image "
                     f"{args.image}^2, eps {args.eps}, grid {G}^2, support "
                     f"{plan.support}, rows sharded over {world} GPU(s), "
                     f"bucketing batches of {plan.batch_vis} visibilities"),
        "mvis_s": modes[best]["mvis_s"],
        "ms_per_step": modes[best]["ms_per_step"],
        "best_mode": best,
        "modes": modes,
        "phases_ms": phases,
        "roofline": roofline,
        "predicted_8gpu": pred,
        # This rank's inputs over PCIe (per GPU; not in mvis_s).
        "h2d_ms": h2d["h2d_ms"],
        "h2d": h2d,
        "pcie_inclusive_mvis_s": round(
            total / ((modes[best]["ms_per_step"] + h2d["h2d_ms"]) * 1e-3)
            / 1e6, 3),
        "steps": args.c3_steps,
        "scaling": "strong",
    }
    del uvw, vis, weight, plan, grid_buf
    torch.cuda.empty_cache()
    return out


def run_wstack(args, torch, dev, world, rank):
    """3-D (w-stacking) ES gridding at the config-2 workload: the same 10M
    rows x 1 channel with w +-500 m, image 5440^2, eps 1e-5 -> grid 8192^2,
    W 8, do_w_stacking (ref sdp_gridder_uvw_es_fft.cpp:578-698): one
    bucketing per call for all w-planes, then per plane the tile scatter
    and the fused FFT with the w-screen; grid and degrid timed separately
    (per GPU; no collective)."""
    from ska_sdp_func.grid_data import GridderUvwEsFft

    uvw, freq, vis, weight, px = make_inputs(
        torch, dev, args.rows, args.chan, args.image, 20251015 + 2 + rank)
    dirty = torch.zeros((args.image, args.image), dtype=torch.float32,
                        device=dev)
    plan = GridderUvwEsFft(uvw, freq, vis, weight, dirty, px, px, args.eps,
                           True)
    plan.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    steps = max(1, args.steps // 2)

    def run(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize(dev)
        t = (time.perf_counter() - t0) / steps
        plan.enable_timing(True)
        fn()
        tm = plan.get_timing()
        plan.enable_timing(False)
        return t, tm

    def grid():
        dirty.zero_()
        plan.grid_uvw_es_fft(uvw, freq, vis, weight, dirty)

    image0 = None
    t_g, tm_g = run(grid)
    image0 = dirty.clone()
    out_vis = torch.zeros_like(vis)
    img = torch.empty_like(dirty)

    def degrid():
        img.copy_(image0)
        plan.ifft_grid_uvw_es(uvw, freq, out_vis, weight, img)

    t_d, tm_d = run(degrid)
    n = args.rows * args.chan
    out = {
        "workload": (f"ES-FFT 3-D (w-stacking), {args.rows} rows x "
                     f"{args.chan} chan, w +-500 m, image {args.image}^2, "
                     f"eps {args.eps}, grid {plan.grid_size}^2, support "
                     f"{plan.support}, {plan.num_w_planes} w-planes"),
        "w_planes": plan.num_w_planes,
        "grid_mvis_s": round(n / t_g / 1e6, 3),
        "grid_ms": round(1e3 * t_g, 3),
        "grid_phases_ms": ({k: round(v, 4) for k, v in tm_g.items()}
                           if tm_g else None),
        "degrid_mvis_s": round(n / t_d / 1e6, 3),
        "degrid_ms": round(1e3 * t_d, 3),
        "degrid_phases_ms": ({k: round(v, 4) for k, v in tm_d.items()}
                             if tm_d else None),
        "steps": steps,
    }
    del uvw, vis, weight, plan, out_vis
    torch.cuda.empty_cache()
    return out


def cpu_baseline_wtower(args, uvw_dev, freq_dev, vis_dev, px):
    """the reference's own CPU imaging gridder on the same
    visibilities -- the C/OpenMP port of sdp_grid_wstack_wtower_grid_all
    (oracle/wtower_port.c, checked against the numpy restatement) on the
    job's host-CPU share, image 8192^2 at the config's pixel size (theta =
    8192 px; the reference has no CPU ES gridder). Every w-stack plane's
    towers are run for every 8th non-empty sub-grid task (hashed) and
    projected to all tasks; the plane FFT + correction is run once and
    counted once per plane."""
    import numpy as np
    import ska_sdp_func.grid_data as g
    from oracle import wtower_port as wp
    cpus = host_cpus()
    threads = wp.set_threads(cpus["usable"])
    N, S, k = 8192, 256, 8
    theta = N * px
    fov = 0.8 * theta
    w_step = g.determine_w_step(theta, fov, 0.0, 0.0)
    H = float(g.determine_max_w_tower_height(
        S, theta, fov, w_step, 8, 16384, 8, 16384, image_size=2 * S,
        subgrid_frac=2.0 / 3.0))
    uvw = uvw_dev.cpu().numpy().astype(np.float64)
    vis = vis_dev.cpu().numpy()
    f = freq_dev.cpu().numpy().astype(np.float64)
    df = float(f[1] - f[0]) if len(f) > 1 else 0.0
    plan = wp.Plan(vis, float(f[0]), df, uvw, N, S, theta, w_step, 8, 16384,
                   8, 16384, 0.0, H)
    t_towers, n_planes, n_vis, done_t, present_t = 0.0, 0, 0, 0, 0
    busiest = None
    for iw in plan.planes():
        t0 = time.perf_counter()
        n_s, done, present = plan.grid_towers(iw, k, 0)
        dt = time.perf_counter() - t0
        if present == 0:
            continue
        n_planes += 1
        t_towers += dt * present / max(done, 1)
        done_t += done
        present_t += present
        if busiest is None or present > busiest[1]:
            busiest = (iw, present)
    image = np.zeros((N, N), np.float32)
    t0 = time.perf_counter()
    plan.finish_plane(busiest[0], image)
    t_plane = time.perf_counter() - t0
    total = args.rows * args.chan
    t_proj = t_towers + n_planes * t_plane
    return {"value": round(total / t_proj / 1e6, 4), "unit": "Mvis/s",
            "cores": threads, "kind": "port",
            "sample": (f"oracle/wtower_port.c (C/OpenMP port of the "
                       f"reference grid_all, {threads} threads) on the "
                       f"config's {total} visibilities, image {N}^2, "
                       f"theta {theta:.4f}, sub-grid {S}, W = W_w = 8, "
                       f"w_step {w_step:.1f}, tower height {H:g}: towers of "
                       f"{done_t} of {present_t} sub-grid tasks over "
                       f"{n_planes} w-stack plane(s), projected "
                       f"{t_towers:.1f} s, + plane FFT/correction "
                       f"{t_plane:.2f} s x {n_planes}")}


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

    from ska_sdp_func.grid_data import GridderUvwEsFft

    uvw, freq, vis, weight, px = make_inputs(
        torch, dev, args.rows, args.chan, args.image, 20251015 + 2 + rank)
    dirty = torch.zeros((args.image, args.image), dtype=torch.float32,
                        device=dev)
    plan = GridderUvwEsFft(uvw, freq, vis, weight, dirty, px, px, args.eps,
                           False)
    plan.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    G, W = plan.grid_size, plan.support
    grid_buf = None
    if world > 1 and args.reduce == "grid":
        grid_buf = torch.empty((G, G), dtype=torch.complex64, device=dev)

    from ska_sdp_func.grid_data.distributed import grid_sharded

    # Multi-GPU, image reduce: two image buffers, so the RCCL reduce of
    # batch k (issued asynchronously, on RCCL's stream) overlaps the
    # kernels of batch k + 1; a buffer's reduce is waited on before the
    # buffer is reused, and every reduce before the timed region ends.
    pipelined = (world > 1 and args.reduce == "image" and
                 not args.no_overlap)
    bufs = [dirty, torch.zeros_like(dirty)] if pipelined else [dirty]
    pending = [None] * len(bufs)
    counter = [0]

    def grid_step():
        k = counter[0] % len(bufs)
        counter[0] += 1
        img = bufs[k]
        if pending[k] is not None:
            pending[k].wait()
            pending[k] = None
        # Fresh image per step (the call accumulates into it).
        img.zero_()
        if world == 1:
            plan.grid_uvw_es_fft(uvw, freq, vis, weight, img)
        elif pipelined:
            pending[k] = grid_sharded(plan, uvw, freq, vis, weight, img,
                                      dist, mode="image", dst=0,
                                      async_op=True)
        else:
            grid_sharded(plan, uvw, freq, vis, weight, img, dist,
                         mode=args.reduce, dst=0, grid_buf=grid_buf)

    def barrier():
        for k, w in enumerate(pending):
            if w is not None:
                w.wait()
                pending[k] = None
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
    ms_per_step = 1e3 * t_grid / args.steps
    total_vis = args.rows * args.chan * world
    value = total_vis * args.steps / t_grid / 1e6

    # Multi-GPU, the other reduce mode: the per-GPU grids summed before one
    # FFT (north star form; 512 MiB per step), timed after the default.
    grid_reduce = None
    if world > 1 and args.reduce == "image" and not args.no_overlap:
        gbuf = torch.empty((G, G), dtype=torch.complex64, device=dev)

        def grid_step_gr():
            dirty.zero_()
            grid_sharded(plan, uvw, freq, vis, weight, dirty, dist,
                         mode="grid", dst=0, grid_buf=gbuf)

        grid_step_gr()
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            grid_step_gr()
        barrier()
        t_gr = time.perf_counter() - t0
        t = torch.tensor([t_gr], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_gr = float(t.item())
        grid_reduce = {"mvis_s": round(total_vis * args.steps / t_gr / 1e6,
                                       3),
                       "ms_per_step": round(1e3 * t_gr / args.steps, 4)}
        del gbuf

    # Per-phase device times (HIP events on the plan stream), in separate
    # calls so that the event synchronisation stays out of the timed loop.
    phase_steps = max(1, min(args.steps, 5))
    plan.enable_timing(True)
    phases = {"bucket": 0.0, "tile_kernel": 0.0, "fft": 0.0, "image": 0.0}
    for _ in range(phase_steps):
        grid_step()
        tm = plan.get_timing()
        for k in phases:
            phases[k] += tm[k] if tm else 0.0
    plan.enable_timing(False)
    barrier()
    avg = {k: v / phase_steps for k, v in phases.items()}

    # Degridding half of the round trip (same image, same step count).
    degrid = None
    if not args.no_degrid:
        image0 = dirty.clone()
        out_vis = torch.zeros_like(vis)
        img = torch.empty_like(dirty)
        for _ in range(args.warmup):
            img.copy_(image0)
            plan.ifft_grid_uvw_es(uvw, freq, out_vis, weight, img)
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            img.copy_(image0)
            plan.ifft_grid_uvw_es(uvw, freq, out_vis, weight, img)
        barrier()
        t_deg = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([t_deg], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            t_deg = float(t.item())
        dph = {"bucket": 0.0, "tile_kernel": 0.0, "fft": 0.0, "image": 0.0}
        plan.enable_timing(True)
        for _ in range(phase_steps):
            img.copy_(image0)
            plan.ifft_grid_uvw_es(uvw, freq, out_vis, weight, img)
            tm = plan.get_timing()
            for k in dph:
                dph[k] += tm[k] if tm else 0.0
        plan.enable_timing(False)
        barrier()
        degrid = {
            "mvis_s": total_vis * args.steps / t_deg / 1e6,
            "ms_per_step": 1e3 * t_deg / args.steps,
            "phases_ms": {k: round(v / phase_steps, 4) for k, v in dph.items()},
        }

    # Host -> device transfer of the config-2 inputs, reported beside the
    # HBM-resident rate.
    h2d = h2d_time(torch, dev, [uvw, vis, weight])

    # Roofline of the dominant kernel of a gridding call.
    kern_bytes = {
        "tile_kernel": scatter_bytes(args.rows, args.chan, G),
        "fft": fft_bytes(G),
        "bucket": args.rows * args.chan * (8 + 4) + args.rows * 12 * 2,
        "image": args.image ** 2 * (8 + 4) + 2 * args.image ** 2 * 4,
    }
    dom = max(avg, key=lambda k: avg[k]) if any(avg.values()) else "tile_kernel"
    achieved = (kern_bytes[dom] / (avg[dom] * 1e-3) / 1e9
                if avg.get(dom) else None)
    kernel_names = {"tile_kernel": "k_scatter_tab (MFMA tile accumulation, "
                                   "LDS tap tables)",
                    "fft": ("k_rows_grid + k_cols_a_grid (pruned FFT passes)"
                            if plan.fused_fft else "rocFFT 2-D C2C inverse"),
                    "bucket": "bucketing (count/scan/fill)",
                    "image": ("k_cols_b_grid (last FFT pass + screen)"
                              if plan.fused_fft else "k_screen_corr_2d")}
    traffic = None
    traffic_src = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
            # Counters were collected at one workload on one build: only
            # reported for that workload and sources hashing to that build.
            wl = pmc.get("_workload", {})
            traffic_src = {"file": "profiles/pmc_traffic.json",
                           "csrc_sha16": pmc.get("_csrc_sha16"),
                           "current_csrc_sha16": csrc_sha16()}
            if (wl.get("rows") == args.rows and wl.get("chan") == args.chan
                    and wl.get("image") == args.image
                    and wl.get("eps") == args.eps
                    and pmc.get("_csrc_sha16") == csrc_sha16()):
                traffic = pmc.get(dom, {}).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    # The same algorithmic bytes over rocprofv3's average duration of the
    # 2-D tile kernel, from the kernel-trace summary committed for this
    # round (profiles/r*_bench_kernel_stats.csv, same config-2 workload).
    rocprof = None
    if dom == "tile_kernel":
        stats = sorted(glob.glob(os.path.join(ROOT, "profiles",
                                              "r*_bench_kernel_stats.csv")))
        if stats:
            try:
                with open(stats[-1]) as f:
                    for r in csv.DictReader(f):
                        if re.search(rf"k_scatter_tab<false, {W + 1}\b",
                                     r["Name"]):
                            avg_ms = float(r["AverageNs"]) * 1e-6
                            gbs = kern_bytes[dom] / (avg_ms * 1e-3) / 1e9
                            rocprof = {
                                "stats_file": os.path.relpath(stats[-1], ROOT),
                                "avg_launch_ms": round(avg_ms, 4),
                                "achieved": round(gbs, 1),
                                "frac": round(gbs / HBM_PEAK_GBS, 4)}
                            break
            except (OSError, ValueError, KeyError):
                rocprof = None

    config3 = None
    if not args.no_config3:
        config3 = run_config3(args, torch, dev, dist, world, rank)
    wstack = None
    if not args.no_wstack:
        wstack = run_wstack(args, torch, dev, world, rank)

    # CPU baselines on rank 0, after every GPU measurement (the other ranks
    # wait at the final barrier). At N > 1 only the like-for-like ES port
    # runs; the w-towers port (~1 min) only at N = 1.
    cpu = None
    cpu_wt = None
    if rank == 0 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args, G, W, plan.beta, G * px)
        except Exception as exc:  # baseline failure must not hide the bench
            cpu = {"value": None, "unit": "Mvis/s", "cores": 0,
                   "kind": "port", "sample": f"failed: {exc!r}"}
        if world > 1 and cpu.get("value"):
            # The job's value is all ranks' visibilities: the CPU baseline
            # is per host (one CPU share), quoted beside it as measured.
            cpu["note"] = (f"one host CPU share; compare with the per-GPU "
                           f"rate {value / world:.1f} Mvis/s or the job's "
                           f"{value:.1f}")
        if world == 1:
            try:
                cpu_wt = cpu_baseline_wtower(args, uvw, freq, vis, px)
            except Exception as exc:
                cpu_wt = {"value": None, "unit": "Mvis/s", "cores": 0,
                          "kind": "port", "sample": f"failed: {exc!r}"}

    if rank == 0:
        line = {
            "metric": "Mvis/s gridded",
            "value": round(value, 3),
            "unit": "Mvis/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (config-2 distribution, generated in HBM)",
            "config": {
                "workload": (f"ES-FFT grid_uvw_es_fft, {args.rows} rows x "
                             f"{args.chan} chan per GPU, image {args.image}^2,"
                             f" eps {args.eps}, grid {G}^2, support {W}, 2-D"),
                "rows_per_gpu": args.rows,
                "channels": args.chan,
                "image_size": args.image,
                "grid_size": G,
                "support": W,
                "epsilon": args.eps,
                "parallelism": (f"row-shard x{world}, RCCL reduce of "
                                f"{args.reduce}" if world > 1 else "1 GPU"),
            },
            "phases_ms": {k: round(v, 4) for k, v in avg.items()},
            "roofline": {
                "kernel": kernel_names[dom],
                "bound": "hbm",
                "achieved": round(achieved, 1) if achieved else None,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                "traffic": traffic,
                "traffic_source": traffic_src,
                # Counter-based view of the same launch: PMC HBM bytes over
                # the event time (the scatter skips empty tiles, so its
                # algorithmic count includes grid bytes it never writes).
                "traffic_GBs": (round(traffic / (avg[dom] * 1e-3) / 1e9, 1)
                                if traffic and avg.get(dom) else None),
                "traffic_frac": (round(traffic / (avg[dom] * 1e-3) / 1e9
                                       / HBM_PEAK_GBS, 4)
                                 if traffic and avg.get(dom) else None),
                "algorithmic_bytes_per_launch": kern_bytes[dom],
                "rocprof": rocprof,
                # SURVEY 8(d) guard: the same launch against the FP32
                # vector / f32-matrix peak (algorithmic flops per vis).
                "fp32_frac": (fp32_roofline(total_vis // world, W,
                                            avg["tile_kernel"])["frac"]
                              if avg.get("tile_kernel") else None),
                "fp32": fp32_roofline(total_vis // world, W,
                                      avg.get("tile_kernel")),
            },
            "call_roofline": {
                "algorithmic_bytes": gridding_bytes(args.rows, args.chan, G,
                                                    args.image),
                "achieved_GBs": round(gridding_bytes(args.rows, args.chan, G,
                                                     args.image)
                                      / (ms_per_step * 1e-3) / 1e9, 1),
                "frac": round(gridding_bytes(args.rows, args.chan, G,
                                             args.image)
                              / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            },
            "degrid": degrid,
            # Inputs resident in HBM when the clock starts; the PCIe copy of
            # one GPU's inputs from pinned host memory is timed separately.
            "h2d_ms": h2d["h2d_ms"],
            "h2d": h2d,
            "pcie_inclusive_mvis_s": round(
                args.rows * args.chan / ((ms_per_step + h2d["h2d_ms"])
                                         * 1e-3) / 1e6, 3),
            "grid_reduce_mode": grid_reduce,
            "config3": config3,
            "wstack_3d": wstack,
            "roundtrip_mvis_s": (round(total_vis / ((ms_per_step
                                                     + degrid["ms_per_step"])
                                                    * 1e-3) / 1e6, 3)
                                 if degrid else None),
            "cpu_baseline": cpu,
            # the reference's CPU imaging gridder (w-towers)
            # on the same visibilities, beside the like-for-like ES port.
            "cpu_baseline_reference_gridder": cpu_wt,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
