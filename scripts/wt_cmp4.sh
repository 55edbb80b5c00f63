#!/bin/bash
# Determinism check: legacy x2, fused x2 on one small case.
set -e
mkdir -p gpurun_out/wt
A="--image 1024 --rows 20000"
SDP_WT_FUSED=0 timeout -k 10 200 python scripts/wt_fused_cmp.py run gpurun_out/wt/l1.npy $A
SDP_WT_FUSED=0 timeout -k 10 200 python scripts/wt_fused_cmp.py run gpurun_out/wt/l2.npy $A
timeout -k 10 200 python scripts/wt_fused_cmp.py run gpurun_out/wt/f1.npy $A
timeout -k 10 200 python scripts/wt_fused_cmp.py run gpurun_out/wt/f2.npy $A
python - <<'PY'
import numpy as np
d = {k: np.load(f"gpurun_out/wt/{k}.npy") for k in ("l1", "l2", "f1", "f2")}
for a, b in (("l1", "l2"), ("f1", "f2"), ("l1", "f1")):
    for bd in (64, 128, 256):
        x, y = d[a][bd:-bd, bd:-bd], d[b][bd:-bd, bd:-bd]
        print(a, b, bd, "max %.3e rms %.3e" % (
            np.abs(x - y).max() / np.abs(x).max(),
            np.sqrt(np.mean((x - y) ** 2) / np.mean(x ** 2))))
PY
rm -f gpurun_out/wt/*.npy
