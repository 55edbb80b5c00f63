"""Generate tests/golden/es_params.json from the REFERENCE's own host code.

Runs oracle/_ref/es_params_probe, built by oracle/ref_build/Makefile straight
from /root/reference/src/ska-sdp-func/grid_data/sdp_gridder_uvw_es_fft_utils.cpp
(ska-sdp-func 1.2.2), over a sweep of image sizes, accuracies and
precisions, and records:
  * grid_size, support, beta/support  (sdp_calculate_params_from_epsilon)
  * Gauss-Legendre quadrature + conv-corr tables for selected plans
    (sdp_generate_gauss_legendre_conv_kernel).
Run from the repo root in the build container:  python tests/golden/make_es_params.py
"""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PROBE = os.path.join(ROOT, "oracle", "_ref", "es_params_probe")


def main():
    subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle", "ref_build")])
    sizes = [64, 100, 128, 240, 255, 256, 512, 840, 1000, 1024, 2048, 4096,
             5440, 8192]
    epsilons = [0.1, 0.05, 1e-2, 1e-3, 1e-4, 1e-5, 3e-6, 1e-6, 1e-7, 1e-8,
                1e-10, 1e-12, 1e-14]
    params = []
    for n in sizes:
        for eps in epsilons:
            for dbl in (0, 1):
                out = subprocess.check_output(
                    [PROBE, "params", str(n), repr(eps), str(dbl)], text=True)
                params.append(json.loads(out))
    tables = []
    picks = {(840, 0.05, 0), (1024, 1e-5, 0), (1024, 1e-12, 1), (256, 1e-5, 0),
             (5440, 1e-5, 0), (128, 1e-10, 1)}
    for p in params:
        if (p["N"], p["eps"], p["double"]) in picks:
            beta = p["beta"] * p["support"]
            out = subprocess.check_output(
                [PROBE, "tables", str(p["N"]), str(p["grid_size"]),
                 str(p["support"]), repr(beta)], text=True)
            tables.append(json.loads(out))
    dst = os.path.join(ROOT, "tests", "golden", "es_params.json")
    with open(dst, "w") as f:
        json.dump({"source": "ska-sdp-func 1.2.2 sdp_gridder_uvw_es_fft_utils.cpp"
                             " via oracle/_ref/es_params_probe",
                   "params": params, "tables": tables}, f, indent=0)
    print(f"wrote {len(params)} params, {len(tables)} tables to {dst}")


if __name__ == "__main__":
    main()
