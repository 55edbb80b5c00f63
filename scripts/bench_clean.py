"""Hogbom CLEAN timing on the GPU: cycles per second at a few image sizes
(dirty image of point sources through a random-uv PSF, threshold below
reach so every cycle runs), with the numpy oracle timed beside it on a
bounded number of cycles.

  python scripts/bench_clean.py [--sizes 256 1024 2048] [--cycles 5000]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func_amd"))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from ska_sdp_func.clean import hogbom_clean
    from oracle import clean_oracle as co
    from tests.test_hogbom_clean import point_dirty, uv_psf
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[256, 1024, 2048])
    ap.add_argument("--cycles", type=int, default=5000)
    ap.add_argument("--cpu-cycles", type=int, default=200)
    ap.add_argument("--ms", action="store_true",
                    help="also time multi-scale CLEAN (5 scales, f64)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    beam = np.array([2.0, 2.0, 1.0, 128.0])
    for n in args.sizes:
        psf64 = uv_psf(n, nbl=200)
        dirty64 = point_dirty(psf64, n)
        for dt, tdt in ((np.float64, torch.float64), (np.float32, torch.float32)):
            d = torch.from_numpy(dirty64.astype(dt)).to(dev)
            p = torch.from_numpy(psf64.astype(dt)).to(dev)
            outs = [torch.zeros((n, n), dtype=tdt, device=dev) for _ in range(3)]
            hogbom_clean(d, p, beam.astype(dt), 0.1, -1e30, 10, *outs)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            hogbom_clean(d, p, beam.astype(dt), 0.1, -1e30, args.cycles, *outs)
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            row = {"n": n, "dtype": np.dtype(dt).name, "cycles": args.cycles,
                   "s": round(t, 4), "us_per_cycle": round(1e6 * t / args.cycles, 2),
                   "GB_s_per_cycle_traffic": round(
                       3 * n * n * np.dtype(dt).itemsize * args.cycles / t / 1e9, 1)}
            if n <= 1024:
                t0 = time.perf_counter()
                co.hogbom_clean(dirty64.astype(dt), psf64.astype(dt), beam, 0.1,
                                -1e30, args.cpu_cycles)
                tc = time.perf_counter() - t0
                row["cpu_oracle_us_per_cycle"] = round(1e6 * tc / args.cpu_cycles, 1)
            print(json.dumps(row), flush=True)
    if args.ms:
        from ska_sdp_func.clean import ms_clean_cornwell
        scales = np.array([0, 2, 4, 8, 16], dtype=np.intc)
        for n in (256, 1024):
            psf64 = uv_psf(n, nbl=200)
            dirty64 = point_dirty(psf64, n)
            d = torch.from_numpy(dirty64).to(dev)
            p = torch.from_numpy(psf64).to(dev)
            outs = [torch.zeros((n, n), dtype=torch.float64, device=dev)
                    for _ in range(3)]
            ms_clean_cornwell(d, p, beam, scales, 0.1, -1e30, 1, *outs)
            torch.cuda.synchronize()              # warm-up (FFT plans)
            t0 = time.perf_counter()
            ms_clean_cornwell(d, p, beam, scales, 0.1, -1e30, 1, *outs)
            torch.cuda.synchronize()
            t_setup = time.perf_counter() - t0    # set-up + one cycle
            t0 = time.perf_counter()
            ms_clean_cornwell(d, p, beam, scales, 0.1, -1e30, args.cycles,
                              *outs)
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            print(json.dumps({"function": "ms_clean_cornwell", "n": n,
                              "scales": 5, "dtype": "float64",
                              "cycles": args.cycles, "s": round(t, 4),
                              "setup_s": round(t_setup, 4),
                              "us_per_cycle": round(
                                  1e6 * (t - t_setup) / args.cycles, 2)}),
                  flush=True)


if __name__ == "__main__":
    main()
