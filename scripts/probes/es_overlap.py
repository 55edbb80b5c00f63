"""Probe: do two half-size ES scatters (bucketing + tile kernel) run faster
concurrently on two streams than one after the other?"""
import sys, time
sys.path[:0] = ["ska-sdp-func_amd", "."]
import numpy as np
import torch
from bench import make_inputs
from ska_sdp_func.grid_data import GridderUvwEsFft

dev = torch.device("cuda:0")
uvw, freq, vis, wt, px = make_inputs(torch, dev, 10_000_000, 1, 5440, 7)
h = 5_000_000
parts = [(uvw[:h], vis[:h], wt[:h]), (uvw[h:], vis[h:], wt[h:])]
dirty = torch.zeros((5440, 5440), dtype=torch.float32, device=dev)
s = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
plans = [GridderUvwEsFft(p[0], freq, p[1], p[2], dirty, px, px, 1e-5, False)
         for p in parts]
G = plans[0].grid_size
grids = [torch.empty((G, G), dtype=torch.complex64, device=dev) for _ in range(2)]
full = GridderUvwEsFft(uvw, freq, vis, wt, dirty, px, px, 1e-5, False)
full.set_stream(s[0].cuda_stream)


def run(concurrent, reps=10):
    for k in range(2):
        plans[k].set_stream(s[k if concurrent else 0].cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for k in range(2):
            plans[k].grid_scatter(parts[k][0], freq, parts[k][1], parts[k][2],
                                  grids[k])
        if concurrent:
            s[0].wait_stream(s[1]); s[1].wait_stream(s[0])
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / reps


def run_full(reps=10):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        full.grid_scatter(uvw, freq, vis, wt, grids[0])
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / reps


for rep in range(3):
    print(f"full call scatter {run_full():.3f} ms, two halves sequential "
          f"{run(False):.3f} ms, two halves concurrent {run(True):.3f} ms",
          flush=True)
for k in range(2):
    plans[k].enable_timing(True)
    plans[k].set_stream(s[0].cuda_stream)
    plans[k].grid_scatter(parts[k][0], freq, parts[k][1], parts[k][2], grids[k])
    print("half", k, plans[k].get_timing())
