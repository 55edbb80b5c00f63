"""The config-4 CPU baseline (oracle/wtower_port.c, a C/OpenMP port of the
reference CPU path of sdp_grid_wstack_wtower_grid_all) agrees with the
numpy restatement (oracle/wtower_oracle.py) before bench_wtower.py times it.

Tolerance: the port grids in complex float (the reference's c64
instantiation), so images agree to 5e-5 of the peak away from a 64-pixel
border, the bound test_wstack_gpu.py uses for the c64 HIP path.
"""
import numpy as np
import scipy.special

import wtower_data as wd
from oracle import wtower_oracle as wo
from oracle import wtower_port as wp

KW = (8, 16384, 8, 16384)


def test_pswf_legendre_series_matches_scipy():
    c = 8 * np.pi / 2
    d = wp.pswf_legendre(c)
    for x in (0.0, 0.1, 0.37, 0.5, 0.81, 0.99):
        val = np.polynomial.legendre.legval(
            x, np.ravel(np.column_stack([d, np.zeros_like(d)])))
        assert abs(val - scipy.special.pro_ang1(0, 0, c, x)[0]) < 1e-12


def test_port_grid_all_matches_oracle():
    case = wd.wstack_case(num_rows=1000, num_chan=3)
    rng = np.random.default_rng(2)
    vis = rng.normal(size=(1000, 3)) + 1j * rng.normal(size=(1000, 3))
    N, S = 256, 64
    args = (case["f0"], case["df"], case["uvw"], S, case["theta"],
            case["w_step"])
    ref = wo.wstack_grid_all(vis, *args, 0.0, 0.0, *KW, 0.0, case["H"],
                             np.zeros((N, N)))
    img = np.full((N, N), 3.0, np.float32)
    wp.set_threads(4)
    n = wp.grid_all(vis.astype(np.complex64), *args, *KW, 0.0, case["H"],
                    img)
    assert n == 3000
    b = 64
    err = (np.abs(img[b:-b, b:-b] - ref[b:-b, b:-b]).max()
           / np.abs(ref[b:-b, b:-b]).max())
    assert err < 5e-5, err
