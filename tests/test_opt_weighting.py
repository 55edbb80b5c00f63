"""Tiled Briggs weighting: sdp_optimized_weighting /
sdp_optimised_indexed_weighting (csrc/visibility/sdp_opt_weighting.hip).

Pins:
  * the reference's own test (tests/visibility/test_opt_weighting.py of
    ska-sdp-func 1.2.2): its input_gen data (8 x 8 identical baselines,
    6 channels, grid 40, robust 2) through count_and_prefix_sum ->
    tiled_indexing / bucket_sort -> the weighting, against the values of
    its reference_briggs_weights (restated in oracle/weighting_oracle.py);
    the reference asserts this for the indexed form;
  * a hand-derived known answer for the per-tile sums (CPU);
  * random multi-tile data: the GPU result against the oracle's per-run
    restatement on the same sorted arrays, 1e-12 relative (cell sums use
    device double atomics, so their rounding order differs).
Semantics and the reference defects not carried over:
include/ska-sdp-func/visibility/sdp_opt_weighting.h.
"""
import ctypes

import numpy as np
import pytest

from oracle import tiled_oracle as to
from oracle import weighting_oracle as wo

TU, TV = 32, 16


def reference_inputs():
    """input_gen of the reference test (:114-245)."""
    freqs = np.array([1e9, 1.1e9, 1.2e9, 1.3e9, 1.4e9, 1.5e9])
    uvw = np.tile(np.array([10.0, 31.0, 21.0]), (8, 8, 1))
    vis = np.full((8, 8, len(freqs), 1), 1j, dtype=complex)
    weights = np.ones((8, 8, len(freqs), 1))
    return dict(uvw=uvw, freqs=freqs, vis=vis, weights=weights, robust=2,
                grid=40, cell=4.06e-5, support=4, max_abs_uv=16011.076569511299)


def _sorted(case, indexed):
    C = len(case["freqs"])
    counts, offsets, _, total = to.count_and_prefix_sum(
        case["uvw"], case["freqs"], C, case["grid"], TU, TV, case["cell"],
        case["support"])
    out, end = to.bucket_sort(
        case["uvw"], case["freqs"], None if indexed else case["vis"],
        None if indexed else case["weights"], case["grid"], TU, TV,
        case["cell"], case["support"], offsets, total, indexed=indexed,
        num_channels=C)
    return counts, offsets, end, total, out


def test_oracle_reproduces_reference_test_expectation():
    case = reference_inputs()
    expect = wo.briggs_global_test_reference(
        case["uvw"], case["freqs"], case["max_abs_uv"], case["grid"],
        case["robust"], case["weights"])
    assert np.allclose(expect, 1.0 / 1.0025)
    _, _, end, total, out = _sorted(case, indexed=True)
    assert total == 384
    got = np.zeros_like(case["weights"])
    wo.opt_briggs_runs(out["uu"], out["vv"], case["weights"], out["tile"],
                       end, case["grid"], case["robust"], got,
                       index=out["vis_index"])
    np.testing.assert_allclose(got, expect, rtol=1e-14)
    _, _, end, _, out = _sorted(case, indexed=False)
    got_b = np.zeros(total)
    wo.opt_briggs_runs(out["uu"], out["vv"], out["weight"], out["tile"], end,
                       case["grid"], case["robust"], got_b)
    np.testing.assert_allclose(got_b, 1.0 / 1.0025, rtol=1e-14)


def test_oracle_known_answer_two_cells():
    """One run, tile (1, 2) of a 64-point grid: three unit weights in one
    cell and a weight of 2 in another, plus an entry from a neighbouring
    tile (listed through its support, not counted). W = 3, 2; sw = 3 * 3 +
    2 = 11; sw2 = 3 * 9 + 4 = 31; R = (5 / 10^0.5)^2 / (31 / 11)."""
    grid = 64
    centre = grid // 2
    top_u = centre - (centre // TU) * TU - TU // 2      # -16
    top_v = centre - (centre // TV) * TV - TV // 2      # -8
    pu, pv = 1, 2
    tile_u, tile_v = pu * TU + top_u, pv * TV + top_v
    cell_a = (tile_u + 5 - centre, tile_v + 3 - centre)
    cell_b = (tile_u + 20 - centre, tile_v + 10 - centre)
    outside = (tile_u - 1 - centre, tile_v + 3 - centre)
    uu = np.array([cell_a[0] + 0.2, cell_a[0] - 0.3, cell_a[0],
                   cell_b[0] + 0.4, outside[0]], float)
    vv = np.array([cell_a[1], cell_a[1] + 0.1, cell_a[1] - 0.49,
                   cell_b[1], outside[1]], float)
    w = np.array([1.0, 1.0, 1.0, 2.0, 5.0])
    code = pv * 32768 + pu
    tiles = np.full(5, code, np.int32)
    offsets = np.array([0, 5] + [5] * 7, np.int32)     # run 0 = entries 0-4
    out = np.full(5, -1.0)
    wo.opt_briggs_runs(uu, vv, w, tiles, offsets, grid, 0.5, out)
    R = (5.0 / 10 ** 0.5) ** 2 / (31.0 / 11.0)
    np.testing.assert_allclose(out[:3], 1.0 / (1 + 3 * R), rtol=1e-15)
    assert out[3] == pytest.approx(2.0 / (1 + 2 * R), rel=1e-15)
    assert out[4] == -1.0                                # not in this tile


def test_library_exports():
    from ska_sdp_func.utility import Lib
    for n in ("sdp_optimized_weighting", "sdp_optimised_indexed_weighting"):
        assert hasattr(Lib.handle(), n)


# ----------------------------------------------------------------- GPU ----

def _gpu_sort(device, case, indexed):
    import torch
    from ska_sdp_func.visibility import (bucket_sort, count_and_prefix_sum,
                                         tiled_indexing)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
    T, B = case["uvw"].shape[:2]
    C = len(case["freqs"])
    g = to.geometry(case["grid"], TU, TV, case["cell"])
    off = torch.zeros(g["ntiles"] + 1, dtype=torch.int32, device=device)
    cnt = torch.zeros(g["ntiles"], dtype=torch.int32, device=device)
    sk = torch.zeros(1, dtype=torch.int32, device=device)
    n = ctypes.c_int(0)
    du, df, dv, dw = (d(case["uvw"]), d(case["freqs"]), d(case["vis"]),
                      d(case["weights"]))
    count_and_prefix_sum(du, df, dv, case["grid"], TU, TV, case["cell"],
                         case["support"], n, off, cnt, sk)
    N = n.value
    mk = lambda dt: torch.zeros(N, dtype=dt, device=device)
    s = dict(uu=mk(torch.float64), vv=mk(torch.float64),
             tile=mk(torch.int32))
    if indexed:
        s["vis_index"] = mk(torch.int32)
        tiled_indexing(du, df, case["grid"], TU, TV, case["cell"],
                       case["support"], C, B, T, s["tile"], s["uu"], s["vv"],
                       s["vis_index"], off)
    else:
        s["weight"] = mk(torch.float64)
        s["vis"] = mk(torch.float64)
        bucket_sort(du, df, dv, dw, case["grid"], TU, TV, case["cell"],
                    case["support"], s["uu"], s["vv"], s["weight"],
                    s["tile"], s["vis"], off)
    return dict(uvw=du, freqs=df, vis=dv, weights=dw, off=off, cnt=cnt,
                n=n, sorted=s)


def _run_gpu(device, case, indexed):
    import torch
    from ska_sdp_func.visibility import (optimised_indexed_weighting,
                                         optimized_weighting)
    g = _gpu_sort(device, case, indexed)
    s = g["sorted"]
    if indexed:
        out = torch.full(case["weights"].shape, -1.0, dtype=torch.float64,
                         device=device)
        optimised_indexed_weighting(
            g["uvw"], g["vis"], g["weights"], case["robust"], case["grid"],
            case["cell"], case["support"], g["n"], s["tile"], s["uu"],
            s["vv"], s["vis_index"], g["off"], g["cnt"], out)
    else:
        out = torch.full((g["n"].value,), -1.0, dtype=torch.float64,
                         device=device)
        optimized_weighting(
            g["uvw"], g["freqs"], g["vis"], g["weights"], case["robust"],
            case["grid"], case["support"], s["uu"], s["vv"], s["weight"],
            s["tile"], g["off"], g["cnt"], out)
    host = {k: v.cpu().numpy() for k, v in s.items()}
    return out.cpu().numpy(), host, g["off"].cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("indexed", [True, False])
def test_gpu_reference_test_case(device, indexed):
    case = reference_inputs()
    out, _, _ = _run_gpu(device, case, indexed)
    if indexed:
        expect = wo.briggs_global_test_reference(
            case["uvw"], case["freqs"], case["max_abs_uv"], case["grid"],
            case["robust"], case["weights"])
        np.testing.assert_allclose(out, expect, rtol=1e-14)
    else:
        np.testing.assert_allclose(out, 1.0 / 1.0025, rtol=1e-14)


def random_case(seed=7):
    rng = np.random.default_rng(seed)
    T, B, C = 4, 90, 5
    uvw = rng.uniform(-12000.0, 12000.0, (T, B, 3))
    # a dense core so that cells collect several visibilities
    uvw[:, :30, :2] *= 0.05
    freqs = 1.0e8 + 1.5e6 * np.arange(C)
    vis = (rng.standard_normal((T, B, C, 1))
           + 1j * rng.standard_normal((T, B, C, 1)))
    weights = rng.uniform(0.5, 2.0, (T, B, C, 1))
    return dict(uvw=uvw, freqs=freqs, vis=vis, weights=weights, robust=-0.5,
                grid=256, cell=1.0e-4, support=3)


@pytest.mark.gpu
@pytest.mark.parametrize("indexed", [True, False])
def test_gpu_random_matches_oracle(device, indexed):
    case = random_case()
    out, s, off = _run_gpu(device, case, indexed)
    if indexed:
        want = np.full(case["weights"].shape, -1.0)
        wo.opt_briggs_runs(s["uu"], s["vv"], case["weights"], s["tile"], off,
                           case["grid"], case["robust"], want,
                           index=s["vis_index"])
    else:
        want = np.full(out.shape, -1.0)
        wo.opt_briggs_runs(s["uu"], s["vv"], s["weight"], s["tile"], off,
                           case["grid"], case["robust"], want)
    written = want != -1.0
    assert written.sum() > 100
    np.testing.assert_array_equal(out == -1.0, ~written)
    np.testing.assert_allclose(out, want, rtol=1e-12)
    assert np.all(out[written] < np.asarray(
        case["weights"] if indexed else s["weight"])[written] + 1e-15)


@pytest.mark.gpu
def test_gpu_errors(device):
    from ska_sdp_func.utility import CError
    from ska_sdp_func.visibility import optimized_weighting
    case = reference_inputs()
    z = np.zeros(4)
    zi = np.zeros(4, np.int32)
    with pytest.raises(CError, match="Error 6"):        # host arrays
        optimized_weighting(case["uvw"], case["freqs"], case["vis"],
                            case["weights"], 2, 40, 4, z, z, z, zi,
                            np.zeros(7, np.int32), zi, z)
    with pytest.raises(CError, match="Error 3"):        # float on host
        optimized_weighting(case["uvw"].astype(np.float32), case["freqs"],
                            case["vis"], case["weights"], 2, 40, 4, z, z, z,
                            zi, np.zeros(7, np.int32), zi, z)
