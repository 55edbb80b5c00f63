"""Throughput of the SURVEY §8(f) rows on one GPU, inputs resident in HBM:
point-source DFT (dft_point_v01), uniform / Briggs weighting, the tiled
Briggs weighting (optimised_indexed_weighting after count_and_prefix_sum +
tiled_indexing) and degrid_uvw_custom, each with the numpy oracle timed
beside it on a bounded slice of the same workload (single-threaded numpy,
kind "port").

  python scripts/bench_next.py [--which dft weighting optw degrid]

Prints one JSON line per function: rate, ms per call, the roofline
quantity (FP64 phasor rate for the DFT, algorithmic HBM bytes for the
others) and the CPU sample rate.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK = 8000.0      # GB/s, MI355X_MICROARCH.md


def timed(fn, sync, reps):
    fn()
    sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    sync()
    return (time.perf_counter() - t0) / reps


def bench_dft(torch, dev, np, reps):
    from ska_sdp_func.visibility import dft_point_v01
    from oracle import dft_oracle as do
    T, B, C, P, S = 16, 8192, 64, 4, 256
    rng = np.random.default_rng(1)
    dirs = rng.uniform(-0.05, 0.05, (S, 3))
    dirs[:, 2] = np.sqrt(1 - dirs[:, 0] ** 2 - dirs[:, 1] ** 2) - 1
    flux = rng.standard_normal((S, C, P)) + 1j * rng.standard_normal((S, C, P))
    uvw = rng.uniform(-5e3, 5e3, (T, B, 3))
    d = [torch.from_numpy(a).to(dev) for a in (dirs, flux, uvw)]
    out = {}
    for name, tdt in (("c128", torch.complex128), ("c64", torch.complex64)):
        vis = torch.zeros((T, B, C, P), dtype=tdt, device=dev)
        t = timed(lambda: dft_point_v01(*d, 100e6, 1e5, vis),
                  torch.cuda.synchronize, reps)
        out[name] = t
    phasors = T * B * C * S
    t0 = time.perf_counter()
    do.dft_point_v01(dirs, flux, uvw[:1, :512], 100e6, 1e5, C, np.complex128)
    tc = time.perf_counter() - t0
    return {"function": "sdp_dft_point_v01", "workload":
            f"{S} sources x {T} times x {B} baselines x {C} channels x {P} pols",
            "ms_per_call_c128": round(1e3 * out["c128"], 3),
            "ms_per_call_c64": round(1e3 * out["c64"], 3),
            "gphasor_s_c128": round(phasors / out["c128"] / 1e9, 2),
            "gphasor_s_c64": round(phasors / out["c64"] / 1e9, 2),
            "bound": "fp64 VALU (double sincos per phasor)",
            "cpu_baseline": {"gphasor_s": round(512 * C * S / tc / 1e9, 5),
                             "cores": 1, "kind": "port",
                             "sample": "oracle dft_point_v01, 1 time x 512 "
                                       "baselines"}}


def bench_weighting(torch, dev, np, reps):
    from ska_sdp_func.visibility import briggs_weights, uniform_weights
    from oracle import weighting_oracle as wo
    T, B, C, P, G = 64, 8192, 64, 4, 4096
    rng = np.random.default_rng(2)
    uvw = rng.uniform(-2e3, 2e3, (T, B, 3))
    freq = 100e6 + 1e5 * np.arange(C)
    max_uv = float(np.abs(uvw[:, :, 0]).max() * freq[-1] / 299792458.0)
    w_in = rng.random((T, B, C, P))
    d_uvw, d_freq, d_in = (torch.from_numpy(a).to(dev) for a in (uvw, freq, w_in))
    grid = torch.zeros((G, G, P), dtype=torch.float64, device=dev)
    w_out = torch.zeros_like(d_in)

    def run_u():
        grid.zero_()
        uniform_weights(d_uvw, d_freq, max_uv, grid, d_in, w_out)

    def run_b():
        grid.zero_()
        briggs_weights(d_uvw, d_freq, max_uv, 0.5, grid, d_in, w_out)
    tu = timed(run_u, torch.cuda.synchronize, reps)
    tb = timed(run_b, torch.cuda.synchronize, reps)
    nv = T * B * C
    # Per visibility: P weights read twice (grid write + read pass) and P
    # written; uvw per (t, b); grid cleared (G^2 P 8) as part of the call.
    bytes_u = nv * P * 8 * 3 + T * B * 24 + G * G * P * 8
    bytes_b = bytes_u + nv * P * 8          # the extra sums pass
    t0 = time.perf_counter()
    sub = slice(0, 2)
    wo.weighting(uvw[sub], freq, max_uv, np.zeros((G, G, P)), w_in[sub],
                 np.zeros_like(w_in[sub]), robust=0.5)
    tc = time.perf_counter() - t0
    return {"function": "sdp_weighting_uniform / _briggs", "workload":
            f"{T} times x {B} baselines x {C} channels x {P} pols, grid {G}^2",
            "ms_per_call_uniform": round(1e3 * tu, 3),
            "ms_per_call_briggs": round(1e3 * tb, 3),
            "gvis_s_uniform": round(nv / tu / 1e9, 2),
            "gvis_s_briggs": round(nv / tb / 1e9, 2),
            "roofline_uniform": {"bound": "hbm", "achieved_GBs": round(bytes_u / tu / 1e9, 1),
                                 "frac": round(bytes_u / tu / 1e9 / HBM_PEAK, 3)},
            "roofline_briggs": {"bound": "hbm", "achieved_GBs": round(bytes_b / tb / 1e9, 1),
                                "frac": round(bytes_b / tb / 1e9 / HBM_PEAK, 3)},
            "cpu_baseline": {"gvis_s": round(2 * B * C / tc / 1e9, 5), "cores": 1,
                             "kind": "port", "sample": "oracle briggs, 2 times"}}


def bench_opt_weighting(torch, dev, np, reps):
    import ctypes
    from ska_sdp_func.visibility import (count_and_prefix_sum,
                                         optimised_indexed_weighting,
                                         tiled_indexing)
    from oracle import weighting_oracle as wo
    T, B, C, P, G, cell, sup = 64, 8192, 64, 1, 4096, 2.0e-5, 4
    rng = np.random.default_rng(4)
    freq = 100e6 + 1e5 * np.arange(C)
    # positions (grid cells) = uvw f / c G cell: a disk reaching 0.45 G
    r = 0.45 * G / (freq[-1] / 299792458.0 * G * cell) * np.sqrt(
        rng.random((T, B)))
    ph = 2 * np.pi * rng.random((T, B))
    uvw = np.stack([r * np.cos(ph), r * np.sin(ph), np.zeros((T, B))], -1)
    w_in = rng.random((T, B, C, P)) + 0.5
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_uvw, d_freq, d_w = d(uvw), d(freq), d(w_in)
    d_vis = torch.zeros((T, B, C, P), dtype=torch.complex128, device=dev)
    ntu, ntv = (G + 31) // 32, (G + 15) // 16
    off = torch.zeros(ntu * ntv + 1, dtype=torch.int32, device=dev)
    cnt = torch.zeros(ntu * ntv, dtype=torch.int32, device=dev)
    sk = torch.zeros(1, dtype=torch.int32, device=dev)
    n = ctypes.c_int(0)
    count_and_prefix_sum(d_uvw, d_freq, d_vis, G, 32, 16, cell, sup, n, off,
                         cnt, sk)
    N = n.value
    tl = torch.zeros(N, dtype=torch.int32, device=dev)
    vi = torch.zeros(N, dtype=torch.int32, device=dev)
    uu = torch.zeros(N, dtype=torch.float64, device=dev)
    vv = torch.zeros(N, dtype=torch.float64, device=dev)
    off0 = off.clone()

    def sort():
        off.copy_(off0)
        tiled_indexing(d_uvw, d_freq, G, 32, 16, cell, sup, C, B, T, tl, uu,
                       vv, vi, off)
    sort()
    offs = off.clone()
    out = torch.zeros_like(d_w)

    def weigh():
        optimised_indexed_weighting(d_uvw, d_vis, d_w, 0.5, G, cell, sup, n,
                                    tl, uu, vv, vi, offs, cnt, out)
    t_sort = timed(sort, torch.cuda.synchronize, reps)
    t_w = timed(weigh, torch.cuda.synchronize, reps)
    nv = T * B * C
    # Per entry: positions 16 B + tile code 4 + index 4, read three times;
    # per visibility one weight read twice (gather) and one written.
    bytes_w = N * (16 + 4 + 4) * 3 + nv * P * 8 * 3
    # CPU: the oracle's per-run loop over the first runs of the same arrays
    h = {k: v.cpu().numpy() for k, v in dict(uu=uu, vv=vv, tl=tl,
                                              vi=vi).items()}
    ho = offs.cpu().numpy()
    k = 0
    while k + 1 < len(ho) and ho[k + 1] - ho[0] < 20000:
        k += 1
    sub = ho.copy()
    sub[k + 1:] = ho[k]
    t0 = time.perf_counter()
    wo.opt_briggs_runs(h["uu"], h["vv"], w_in, h["tl"], sub, G, 0.5,
                       np.zeros_like(w_in), index=h["vi"])
    tc = time.perf_counter() - t0
    return {"function": "sdp_optimised_indexed_weighting", "workload":
            f"{T} times x {B} baselines x {C} channels, grid {G}^2, tiles "
            f"32 x 16, support {sup}: {N} tile entries",
            "ms_per_call_weighting": round(1e3 * t_w, 3),
            "ms_per_call_tiled_indexing": round(1e3 * t_sort, 3),
            "gvis_s_weighting": round(nv / t_w / 1e9, 2),
            "roofline_weighting": {"bound": "hbm", "achieved_GBs":
                                   round(bytes_w / t_w / 1e9, 1),
                                   "frac": round(bytes_w / t_w / 1e9
                                                 / HBM_PEAK, 3)},
            "cpu_baseline": {"mentries_s": round(int(ho[k] - ho[0]) / tc
                                                 / 1e6, 4),
                             "cores": 1, "kind": "port",
                             "sample": f"oracle per-run loop, {k} runs"}}


def bench_degrid(torch, dev, np, reps):
    from ska_sdp_func.grid_data import degrid_uvw_custom
    from oracle import degrid_custom_oracle as dco
    T, B, C, P, X, Z, K, KW, OS = 32, 8192, 16, 4, 1024, 4, 8, 4, 16000
    rng = np.random.default_rng(3)
    d_grid = (torch.randn((C, Z, X, X, P), dtype=torch.complex128, device=dev))
    uvw = rng.uniform(-1500.0, 1500.0, (T, B, 3))
    ku, kw = rng.random((OS, K)), rng.random((OS, KW))
    d = [torch.from_numpy(a).to(dev) for a in (uvw, ku, kw)]
    vis = torch.zeros((T, B, C, P), dtype=torch.complex128, device=dev)
    args = (0.1, 250.0, 100e6, 0.1e6, False)
    t = timed(lambda: degrid_uvw_custom(d_grid, *d, *args, vis),
              torch.cuda.synchronize, reps)
    nv = T * B * C
    grid_np = d_grid[:, :, :, :, :].cpu().numpy()
    ref = np.zeros((1, 256, C, P), complex)
    t0 = time.perf_counter()
    dco.degrid(grid_np, uvw[:1, :256], ku, kw, *args, ref)
    tc = time.perf_counter() - t0
    # Algorithmic: vis written (16 P B), uvw; taps gathered from L2 count
    # as K^2 KW cells of 16 P B each.
    return {"function": "sdp_degrid_uvw_custom", "workload":
            f"{T} times x {B} baselines x {C} channels x {P} pols, grid "
            f"[{C}][{Z}][{X}][{X}][{P}] c128, K {K}, KW {KW}",
            "ms_per_call": round(1e3 * t, 3), "mvis_s": round(nv / t / 1e6, 1),
            "tap_gather_GBs": round(nv * K * K * KW * 16 * P / t / 1e9, 1),
            "bound": "L2 gather (K^2 KW taps per visibility)",
            "cpu_baseline": {"mvis_s": round(256 * C / tc / 1e6, 4), "cores": 1,
                             "kind": "port", "sample": "oracle, 1 time x 256 baselines"}}


def main():
    import numpy as np
    import torch
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", nargs="+",
                    default=["dft", "weighting", "optw", "degrid"])
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    fns = {"dft": bench_dft, "weighting": bench_weighting,
           "optw": bench_opt_weighting, "degrid": bench_degrid}
    for w in args.which:
        print(json.dumps(fns[w](torch, dev, np, args.reps)), flush=True)


if __name__ == "__main__":
    main()
