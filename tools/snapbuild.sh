#!/bin/bash
# Build libraocp_hip.so from a snapshot of the sources (edits made while hipcc runs cannot
# reach one of its two passes): tools/snapbuild.sh <tag> -> /tmp/libraocp_hip_<tag>.so
set -e
tag=$1
root=$(cd "$(dirname "$0")/.." && pwd)
snap=/tmp/snap_$tag
rm -rf "$snap" && mkdir -p "$snap/raocp-toolbox_amd" "$snap/include"
cp -r "$root/raocp-toolbox_amd/csrc" "$snap/raocp-toolbox_amd/"
cp "$root/include/raocp_hip.h" "$snap/include/"
cd "$snap/raocp-toolbox_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -shared csrc/raocp_capi.hip -o /tmp/libraocp_hip_$tag.so
