"""Turn FETCH_SIZE / WRITE_SIZE passes into per-phase HBM bytes per launch.

Usage: python scripts/pmc_traffic.py OUTDIR [profiles/pmc_traffic.json]

Counters are in KiB per dispatch. On gfx950 FETCH_SIZE reports half the
bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM section), so
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024. Every kernel of a phase
(bench.py phases: bucket, tile_kernel, fft, image) is summed over its
dispatches and divided by the number of calls profiled (= dispatches of
the tile kernel), giving bytes per call of that phase.
"""
import collections
import csv
import glob
import json
import os
import re
import sys

PHASES = {
    "bucket": ("k_bucket_count", "k_scan_columns", "k_scan_bins",
               "k_bucket_fill", "k_zero_shared_tiles"),
    "tile_kernel": ("k_scatter_tab", "k_scatter_mfma", "k_scatter<",
                    "k_scatter(", "k_gather_tab", "k_gather_mfma", "k_gather<",
                    "k_gather("),
    "image": ("k_screen_corr_2d", "k_screen_accumulate", "k_apply_correction",
              "k_reverse_screen", "k_cols_b_grid", "k_cols_b_herm"),
    # fused FFT passes (es_fft.hip); rocFFT kernels match "fft" below
    "fft": ("k_rows_grid", "k_cols_a_grid", "k_rows_herm", "k_cols_a_herm",
            "k_row_occupancy"),
}


def phase_of(name):
    for ph, keys in PHASES.items():
        if any(k in name for k in keys):
            return ph
    if "rocfft" in name.lower() or "fft" in name.lower() or "transpose" in name.lower():
        return "fft"
    return None


def load(outdir, ctr):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(outdir, ctr, "**", "*counter_collection.csv"),
                       recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != ctr:
                    continue
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def main():
    outdir = sys.argv[1]
    dst = sys.argv[2] if len(sys.argv) > 2 else None
    fetch, write = load(outdir, "FETCH_SIZE"), load(outdir, "WRITE_SIZE")
    res = collections.defaultdict(lambda: {"fetch_kib": 0.0, "write_kib": 0.0,
                                           "kernels": {}})
    # Calls of the path = dispatches of its tile kernel (one per call).
    calls = max(len(v) for k, v in fetch.items()
                if phase_of(k) == "tile_kernel")
    for name in sorted(set(fetch) | set(write)):
        ph = phase_of(name)
        if ph is None:
            continue
        # Per call: a kernel may run several times per call (rocFFT passes).
        f = sum(fetch.get(name, [])) / calls
        w = sum(write.get(name, [])) / calls
        m = re.search(r"\b(k_[a-z_0-9]+(<[^>]*>)?)", name)
        short = m.group(1) if m else name.split("(")[0][-80:]
        res[ph]["fetch_kib"] += f
        res[ph]["write_kib"] += w
        res[ph]["kernels"][short] = {"fetch_kib": f, "write_kib": w,
                                     "dispatches_per_call": len(fetch.get(name, [])) / calls}
    sys.path.insert(0, os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))))
    from bench import csrc_sha16
    out = {"_calls": calls,
           # The build the counters describe: bench.py reports the traffic
           # only while the sources hash to this value.
           "_csrc_sha16": csrc_sha16(),
           # bench.py reports the traffic only for this workload (the bench
           # arguments the counters were collected with; defaults here).
           "_workload": {"rows": 10000000, "chan": 1, "image": 5440,
                         "eps": 1e-5}}
    for ph, r in res.items():
        r["hbm_bytes_per_launch"] = int((2 * r["fetch_kib"] + r["write_kib"]) * 1024)
        out[ph] = r
    out["_note"] = ("(2*FETCH_SIZE + WRITE_SIZE) KiB * 1024 per launch of the "
                    "phase; FETCH doubled per MI355X_MICROARCH.md gfx950 note")
    txt = json.dumps(out, indent=1)
    print(txt)
    if dst:
        with open(dst, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
