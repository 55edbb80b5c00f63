#!/bin/bash
# Per-kernel register / spill / LDS figures of one source file for gfx950:
#   scripts/kstats.sh csrc/grid_data/es_fft.hip [kernel-name-regex]
# (compiles with --save-temps into /tmp/kst and reads the AMDGPU metadata)
set -e
SRC=$1; PAT=${2:-.}
cd "$(dirname "$0")/../ska-sdp-func_amd"
D=/tmp/kst/$(basename "$SRC")
mkdir -p "$D"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 \
    -munsafe-fp-atomics $KFLAGS -I../include -Icsrc -x hip -c "$SRC" \
    --save-temps=obj -o "$D/out.o" 2> /dev/null || \
  (cd "$D" && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 \
    -munsafe-fp-atomics -I"$OLDPWD/../include" -I"$OLDPWD/csrc" -x hip -c \
    "$OLDPWD/$SRC" --save-temps -o out.o)
S=$(ls "$D"/*gfx950*.s 2>/dev/null | head -1)
[ -z "$S" ] && S=$(ls ./*gfx950*.s | head -1)
python3 - "$S" "$PAT" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
pat = re.compile(sys.argv[2])
for m in re.finditer(r"\.name:\s+(\S+)\n(.*?)(?=\n  - \.|\Z)", txt, re.S):
    name, body = m.group(1), m.group(2)
    if not pat.search(name):
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", body) or [None, "?"])[1]
    print(f"{name[:110]}: vgpr {g('vgpr_count')} agpr {g('agpr_count')} "
          f"sgpr {g('sgpr_count')} vspill {g('vgpr_spill_count')} "
          f"sspill {g('sgpr_spill_count')} lds {g('group_segment_fixed_size')}")
PY
