#!/bin/bash
# Per-kernel VGPR / scratch / occupancy of one HIP source (gfx950).
# Usage: scripts/kres.sh path/to/file.hip [extra hipcc flags]
SRC=$1; shift
case "$SRC" in
  *es_kernels.hip|*sdp_grid_wstack_wtower.hip) VGPR_FORM="-mllvm -amdgpu-mfma-vgpr-form" ;;
esac
ROOT=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics \
    -I"$ROOT/include" -I"$ROOT/ska-sdp-func_amd/csrc" $VGPR_FORM -x hip -c "$SRC" -o /tmp/kres.o \
    -Rpass-analysis=kernel-resource-usage "$@" 2>&1 | python3 -c '
import re, sys, subprocess
cur = None; rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = subprocess.run(["c++filt"], input=m.group(1), capture_output=True, text=True).stdout.strip()
        name = re.sub(r"sdp_es::\(anonymous namespace\)::", "", name)
        name = re.sub(r"HIP_vector_type<float, 2u>", "float2", name)
        cur = {"name": name[:90]}; rows.append(cur); continue
    for key, pat in (("vgpr", r" VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur is not None: cur[key] = int(m.group(1))
    if "error" in line: print(line.rstrip())
for r in rows:
    print("%-92s v%4d a%4d scr%5d occ%2d" % (r["name"], r.get("vgpr", 0), r.get("agpr", 0), r.get("scratch", 0), r.get("occ", 0)))
'
