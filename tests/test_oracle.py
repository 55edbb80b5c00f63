"""CPU tests of the oracle itself (no GPU).

The oracle is the checker for every GPU parity test, so it is pinned here:
  1. its parameter maths == the REFERENCE's own host code, run here
     (tests/golden/es_params.json from oracle/_ref; exact equality);
  2. its dirty image == a direct DFT of the same visibilities, to the
     kernel's accuracy (2-D and 3-D, f32 taps and f64 taps);
  3. its degridder == the adjoint DFT, and grid/degrid are adjoint
     (the reference's own adjointness test recipe).
"""
import json
import os

import numpy as np
import pytest

from es_data import make_case, reference_test_case, rel_l2
from oracle import es_oracle, es_params

HERE = os.path.dirname(os.path.abspath(__file__))


def _golden():
    with open(os.path.join(HERE, "golden", "es_params.json")) as f:
        return json.load(f)


def test_params_match_reference_golden():
    gold = _golden()["params"]
    assert len(gold) > 300
    for p in gold:
        g, w, b = es_params.params_from_epsilon(p["eps"], p["N"],
                                                bool(p["double"]))
        assert (g, w) == (p["grid_size"], p["support"]), p
        assert b == p["beta"], p


def test_quadrature_tables_match_reference_golden():
    for t in _golden()["tables"]:
        qk, qn, qw, cc, _ = es_params.gauss_legendre_conv_kernel(
            t["N"], t["G"], t["W"], t["beta"])
        np.testing.assert_allclose(qn, t["quad_nodes"], rtol=0, atol=1e-15)
        np.testing.assert_allclose(qw, t["quad_weights"], rtol=1e-13,
                                   atol=1e-16)
        np.testing.assert_allclose(qk, t["quad_kernel"], rtol=1e-13,
                                   atol=1e-300)
        np.testing.assert_allclose(cc, t["conv_corr"], rtol=1e-12)


def test_good_size():
    for n, want in [(1, 1), (12, 12), (13, 14), (97, 98), (521, 525),
                    (841, 847), (4097, 4116)]:
        assert es_params.good_size_complex(n) == want


@pytest.mark.parametrize("dbl,do_w,eps,tol", [
    (True, False, 1e-10, 1e-9),
    (False, False, 1e-5, 2e-5),
    (True, True, 1e-10, 1e-9),
    (False, True, 1e-5, 5e-5),   # f32 phasor + taps
])
def test_oracle_grid_matches_dft(dbl, do_w, eps, tol):
    n = 96
    uvw, freq, vis, wt, px = make_case(21, 150, 2, n, dbl=dbl,
                                       w_range=300.0)
    dirty0 = np.zeros((n, n), np.float64 if dbl else np.float32)
    geo = es_oracle.geometry_for(uvw, freq, vis, dirty0, px, eps, do_w)
    out = es_oracle.grid_uvw_es_fft(geo, uvw, freq, vis, wt, dirty0)
    ref = es_oracle.dft_dirty(uvw, freq, vis, wt, n, px, do_w)
    assert rel_l2(out, ref) < tol


@pytest.mark.parametrize("dbl,do_w,eps,tol", [
    (True, False, 1e-10, 1e-9),
    (True, True, 1e-10, 1e-9),
    (False, False, 1e-5, 2e-5),
])
def test_oracle_degrid_matches_dft(dbl, do_w, eps, tol):
    n = 64
    uvw, freq, vis, wt, px = make_case(22, 60, 2, n, dbl=dbl, w_range=300.0)
    rng = np.random.default_rng(1)
    dirty = rng.standard_normal((n, n)).astype(np.float64 if dbl
                                                else np.float32)
    geo = es_oracle.geometry_for(uvw, freq, vis, dirty, px, eps, do_w)
    # The degridder first divides the image by the correction; the DFT
    # reference takes the raw image.
    out, _ = es_oracle.ifft_degrid_uvw_es(geo, uvw, freq, dirty)
    ref = es_oracle.dft_degrid(uvw, freq, dirty.astype(np.float64), px, do_w)
    assert rel_l2(out, ref) < tol


@pytest.mark.parametrize("do_single,do_w", [(True, False), (False, False),
                                            (False, True)])
def test_oracle_adjointness_reference_recipe(do_single, do_w):
    """test_gridder_uvw_es_fft.py:413-518 of the reference, on the oracle,
    at the reference's own sizes (1000 rows x 10 channels, 1024^2)."""
    uvw, freqs, tvis, wt, tdirty, px = reference_test_case(do_single)
    geo = es_oracle.geometry_for(uvw, freqs, tvis, tdirty, px, 1e-5, do_w)
    dirty = es_oracle.grid_uvw_es_fft(geo, uvw, freqs, tvis, wt,
                                      np.zeros_like(tdirty))
    adj1 = np.vdot(dirty, tdirty)
    vis, _ = es_oracle.ifft_degrid_uvw_es(geo, uvw, freqs, tdirty)
    adj2 = np.vdot(vis, tvis.astype(np.complex128)).real
    err = abs(adj1 - adj2) / max(abs(adj1), abs(adj2))
    assert err < (1e-5 if do_single else 1e-12)


@pytest.mark.parametrize("dbl,do_w", [(False, False), (True, False),
                                      (False, True), (True, True)])
def test_parallel_scatter_equals_serial(dbl, do_w):
    """The stripe-parallel oracle scatter used by the full-size parity tests
    (oracle_es_grid_*_par) is bit-identical to the serial restatement:
    same taps, same per-cell summation order."""
    n = 200
    uvw, freq, vis, wt, px = make_case(31, 3000, 3, n, dbl=dbl,
                                       w_range=300.0, frac=0.49)
    dirty0 = np.zeros((n, n), np.float64 if dbl else np.float32)
    geo = es_oracle.geometry_for(uvw, freq, vis, dirty0, px, 1e-5, do_w)
    L = es_oracle.lib()
    ser = es_oracle.lib().oracle_es_grid_f64 if dbl else L.oracle_es_grid_f32
    par = L.oracle_es_grid_f64_par if dbl else L.oracle_es_grid_f32_par
    G = geo["grid_size"]
    beta, uvs, ws, mpw = es_oracle._precision_args(geo, dbl)
    p = es_oracle._ptr
    for plane in range(min(geo["num_w_planes"], 3)):
        a = np.zeros((G, G), np.complex128)
        b = np.zeros((G, G), np.complex128)
        args = (len(uvw), 3, p(uvw), p(freq), p(vis), p(wt), G,
                geo["support"], beta, uvs, ws, mpw, int(do_w), plane)
        ser(*args, p(a))
        par(*args, p(b))
        assert np.array_equal(a, b)
        assert np.count_nonzero(a) > 0
