#!/bin/bash
# Kernel resource metadata (VGPRs, AGPRs, spills, scratch, LDS) of the built library's gfx950
# code objects: tools/kmeta.sh [kernel-name-regex]. The library links several HIP translation
# units (raocp_capi, raocp_dynr, raocp_cp4): its .hip_fatbin section holds one offload bundle
# per unit, each unbundled here.
set -e
LIB=${LIB:-/root/repo/raocp-toolbox_amd/raocp/core/libraocp_hip.so}
D=$(mktemp -d)
objcopy --dump-section .hip_fatbin=$D/fat.bin "$LIB"
python3 - "$D" <<'PY'
import sys
d = sys.argv[1]
data = open(f"{d}/fat.bin", "rb").read()
magic = b"__CLANG_OFFLOAD_BUNDLE__"
offs = []
i = data.find(magic)
while i >= 0:
    offs.append(i)
    i = data.find(magic, i + 1)
offs.append(len(data))
for n in range(len(offs) - 1):
    open(f"{d}/b{n}.bin", "wb").write(data[offs[n]:offs[n + 1]])
PY
: > $D/notes.txt
for b in $D/b*.bin; do
  if /opt/rocm/llvm/bin/clang-offload-bundler --type=o --unbundle --input=$b \
       --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$b.co 2>/dev/null; then
    /opt/rocm/llvm/bin/llvm-readelf --notes $b.co >> $D/notes.txt 2>/dev/null || true
  fi
done
python3 - "$D/notes.txt" "${1:-.}" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
pat = re.compile(sys.argv[2])
for blk in txt.split("  - .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if not pat.search(name): continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
    agpr = blk.split("\n")[0].strip(": ")
    print(f"{name[:90]:90s} vgpr {g('vgpr_count'):>4} agpr {agpr:>4} vspill {g('vgpr_spill_count'):>3} scratch {g('private_segment_fixed_size'):>5} lds {g('group_segment_fixed_size'):>6}")
PY
rm -rf $D
