"""Host-side arithmetic of the bench lines (no GPU): the roofline objects
bench_wtower.py attaches to the config-4 line, and bench.py's source hash
that ties profiles/pmc_traffic.json to the build it was measured on."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_wtower_image_side_roofline():
    import bench_wtower as bw
    G = 16384
    # 873 ms per call, 642.6 ms of it in the tower kernels, 32 planes.
    r = bw.image_side(873.0, {"kernel_ms": 642.6, "launches": 32}, 32, G)
    assert r["bound"] == "hbm" and r["unit"] == "GB/s"
    assert r["ms_per_plane"] == pytest.approx((873.0 - 642.6) / 32, abs=1e-3)
    assert r["algorithmic_bytes_per_plane"] == 7.0 * G * G * 8
    achieved = 7.0 * G * G * 8 / ((873.0 - 642.6) / 32 * 1e-3) / 1e9
    assert r["achieved"] == pytest.approx(achieved, rel=1e-3)
    assert r["frac"] == pytest.approx(achieved / bw.HBM_PEAK_GBS, rel=1e-3)
    # No timing, no planes, or towers longer than the call: no roofline.
    assert bw.image_side(873.0, None, 32, G) is None
    assert bw.image_side(873.0, {"kernel_ms": 1.0, "launches": 0}, 32, G) is None
    assert bw.image_side(873.0, {"kernel_ms": 1.0, "launches": 1}, 0, G) is None
    assert bw.image_side(10.0, {"kernel_ms": 20.0, "launches": 1}, 1, G) is None


def test_wtower_tower_roofline():
    import bench_wtower as bw
    tm = {"kernel_ms": 640.0, "launches": 32, "vis": 10_000_000,
          "layers": 400_000, "subgrid_size": 256}
    r = bw.roofline(tm, "k_tower_dft")
    flops = 8.0 * 256 ** 2 * (tm["vis"] + tm["layers"]) / 32
    assert r["algorithmic_flops_per_launch"] == flops
    assert r["achieved"] == pytest.approx(flops / 0.020 / 1e12, rel=1e-3)
    assert r["bound"] == "mfma" and r["frac"] <= 1.0


def test_pmc_traffic_is_stamped_with_the_sources():
    import json
    import bench
    h = bench.csrc_sha16()
    assert len(h) == 16 and int(h, 16) >= 0
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
        pmc = json.load(f)
    # The committed counters describe the committed sources (bench.py
    # reports them only on a match).
    assert pmc["_csrc_sha16"] == h
    assert "k_scan_bins" not in json.dumps(pmc)
    for ph in ("bucket", "tile_kernel", "fft", "image"):
        assert pmc[ph]["hbm_bytes_per_launch"] > 0
