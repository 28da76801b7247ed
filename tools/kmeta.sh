#!/bin/bash
# Kernel resource metadata (VGPRs, AGPRs, spills, scratch, LDS) of the built library's gfx950
# code object: tools/kmeta.sh [kernel-name-regex]
set -e
LIB=${LIB:-/root/repo/raocp-toolbox_amd/raocp/core/libraocp_hip.so}
D=$(mktemp -d)
objcopy --dump-section .hip_fatbin=$D/fat.bin "$LIB"
/opt/rocm/llvm/bin/clang-offload-bundler --type=o --unbundle --input=$D/fat.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$D/gfx950.co
/opt/rocm/llvm/bin/llvm-readelf --notes $D/gfx950.co > $D/notes.txt
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
