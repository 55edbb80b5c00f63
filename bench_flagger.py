#!/usr/bin/env python3
"""Benchmark of the HIP dynamic-threshold flagger at SURVEY.md section 8(d)
config 5: vis [518, 19306, 1024, 1] complex64 (1.02e10 visibilities,
82 GB) with planted RFI, flags int32 (41 GB), alpha 0.5, thresholds 3.5,
sampling step 1, window 0, median history 20, one MI355X.

Prints one JSON line (same field layout as bench.py). Inputs are generated
in HBM; a "step" is one sdp_flagger_dynamic_threshold call over the whole
array. Roofline: HBM, on the bytes the kernel moves: the visibility read
(8 B, c64) plus a 4 B flag store only where a flag is raised (the kernel
writes no flag for an unflagged visibility; the caller's zeroed buffer
stands), i.e. 8 + 4 f B per visibility at flagged fraction f. The SURVEY
8(d) figure of 12 B per visibility (every flag written) is reported beside
it as "frac_survey_12B". The CPU baseline runs the oracle
(oracle/flagger_oracle.c, OpenMP) on a bounded sample of baselines.

  python bench_flagger.py [--T 518 --B 19306 --C 1024 --P 1 --steps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=518)
    ap.add_argument("--B", type=int, default=19306)
    ap.add_argument("--C", type=int, default=1024)
    ap.add_argument("--P", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("--step", type=int, default=1)
    ap.add_argument("--dtype", choices=("c64", "c128"), default="c64")
    ap.add_argument("--cpu-sample-baselines", type=int, default=256)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def make_vis(torch, dev, T, B, C, P, seed, dtype):
    """1+1j + 0.05 complex noise, planted narrowband / broadband RFI,
    generated time step by time step in HBM."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    vis = torch.empty((T, B, C, P), dtype=dtype, device=dev)
    real = torch.float32 if dtype == torch.complex64 else torch.float64
    for t in range(T):
        re = torch.randn((B, C, P), generator=g, device=dev,
                         dtype=real) * 0.05 + 1.0
        im = torch.randn((B, C, P), generator=g, device=dev,
                         dtype=real) * 0.05 + 1.0
        vis[t] = torch.complex(re, im)
    n_nb = max(1, T * B * P // 20)
    idx = [torch.randint(0, n, (n_nb,), generator=g, device=dev)
           for n in (T, B, C, P)]
    vis[idx[0], idx[1], idx[2], idx[3]] += 20.0
    nb = max(1, B // 3)
    tt = torch.randint(1, T, (nb,), generator=g, device=dev)
    bb = torch.randint(0, B, (nb,), generator=g, device=dev)
    vis[tt, bb] *= 5.0
    return vis


def cpu_baseline(vis_dev, args, kw):
    import numpy as np
    from oracle import flagger_oracle as fo

    from bench import host_cpus

    host = host_cpus()
    # at least 8 baselines per thread, so that every thread has work
    nb = min(args.B, max(args.cpu_sample_baselines, 8 * host["usable"]))
    sample = np.ascontiguousarray(vis_dev[:, :nb].cpu().numpy())
    flags = np.zeros(sample.shape, np.int32)
    threads = fo.lib().oracle_flagger_set_threads(host["usable"])
    t0 = time.perf_counter()
    fo.flagger_dynamic_threshold(sample, flags, **kw)
    dt = time.perf_counter() - t0
    return {"value": round(sample.size / dt / 1e6, 3), "unit": "Mvis/s",
            "cores": threads, "host_cpus": host, "kind": "port",
            "sample": (f"oracle/flagger_oracle.c (OpenMP over baselines) on "
                       f"{nb} of {args.B} baselines x {args.T} x {args.C} x "
                       f"{args.P} ({dt:.2f} s), {threads} threads = the CPUs "
                       f"this job may use of the host's {host['nproc']}")}


def main():
    args = parse()
    import torch
    from ska_sdp_func.visibility import flagger_dynamic_threshold

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    cdt = torch.complex64 if args.dtype == "c64" else torch.complex128
    vis = make_vis(torch, dev, args.T, args.B, args.C, args.P, 20251015 + 5,
                   cdt)
    flags = torch.zeros(vis.shape, dtype=torch.int32, device=dev)
    kw = dict(alpha=0.5, threshold_magnitudes=3.5, threshold_variations=3.5,
              threshold_broadband=3.5, sampling_step=args.step,
              window=args.window, window_median_history=20)
    for _ in range(args.warmup):
        flagger_dynamic_threshold(vis, flags, **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        flagger_dynamic_threshold(vis, flags, **kw)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    n = vis.numel()
    value = n / dt / 1e6
    flagged = float(flags.sum(dtype=torch.int64).item()) / n
    # Bytes moved: every visibility read, a flag stored where raised.
    algo = int(round(vis.element_size() * n + 4 * flagged * n))
    achieved = algo / dt / 1e9
    survey = (vis.element_size() + 4) * n   # every flag written
    survey_gbs = survey / dt / 1e9
    cpu = None if args.no_cpu_baseline else cpu_baseline(vis, args, kw)
    line = {
        "metric": "Mvis/s flagged",
        "value": round(value, 3),
        "unit": "Mvis/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": f"{args.dtype} in, f64 statistics, int32 flags",
        "data": "synthetic (config-5 shape, planted RFI, generated in HBM)",
        "config": {"workload": (f"sdp_flagger_dynamic_threshold vis "
                                f"[{args.T}, {args.B}, {args.C}, {args.P}] "
                                f"{args.dtype}, step {args.step}, window "
                                f"{args.window}, history 20"),
                   "flagged_fraction": round(flagged, 5)},
        "roofline": {"kernel": "k_flagger (wave per baseline stream)",
                     "bound": "hbm", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": None,
                     "algorithmic_bytes_per_launch": algo,
                     "bytes_model": (f"{vis.element_size()} B read per "
                                     f"visibility + 4 B flag store x "
                                     f"flagged fraction {flagged:.5f}"),
                     "achieved_survey_12B": round(survey_gbs, 1),
                     "frac_survey_12B": round(survey_gbs / HBM_PEAK_GBS, 4)},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
