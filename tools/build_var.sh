#!/bin/bash
# Variant builds of the library for A/B timing on the GPU box (RAOCP_HIP_LIB=build/var/<name>.so):
#   tools/build_var.sh <name> "<-D flags for raocp_capi.hip>" [<name> "<flags>" ...]
# Each variant recompiles the capi translation unit (the L / L^T kernels live there) and links
# it with the current objects of the other translation units; the builds run in parallel.
set -e
cd "$(dirname "$0")/../raocp-toolbox_amd"
mkdir -p ../build/var
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $flags \
      -c csrc/raocp_capi.hip -o ../build/var/capi_$name.o > ../build/var/$name.build.txt 2>&1 &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared ../build/var/capi_$name.o ../build/obj/raocp_dynr.o \
      ../build/obj/raocp_cp4.o ../build/obj/raocp_cp5.o ../build/obj/raocp_dyn4.o -o ../build/var/$name.so &&
    echo "variant $name built" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
