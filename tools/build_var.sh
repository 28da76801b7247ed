#!/bin/bash
# Variant builds of the library for A/B timing on the GPU box (RAOCP_HIP_LIB=build/var/<name>.so):
#   tools/build_var.sh <name> "<-D flags for raocp_capi.hip>" [<name> "<flags>" ...]
# Each variant recompiles the capi translation unit (the L / L^T kernels live there) and links
# it with the current objects of the other translation units; the builds run in parallel.
# VAR_ALL=1: every translation unit with the variant's flags (e.g. -DRAOCP_DIAG).
# VAR_UNIT=<u> (dynr, cp4, cp5): only that unit with the flags, linked with the current
# objects of the others (capi included): a one-minute build.
set -e
cd "$(dirname "$0")/../raocp-toolbox_amd"
mkdir -p ../build/var
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  ( others="../build/obj/raocp_dynr.o ../build/obj/raocp_cp4.o ../build/obj/raocp_cp5.o"
    if [ -n "${VAR_UNIT:-}" ]; then
      objs="../build/obj/raocp_capi.o"
      for u in dynr cp4 cp5; do
        if [ "$u" = "$VAR_UNIT" ]; then
          /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $flags \
            -c csrc/raocp_$u.hip -o ../build/var/${u}_$name.o > ../build/var/$name.build.txt 2>&1 || exit 1
          objs="$objs ../build/var/${u}_$name.o"
        else
          objs="$objs ../build/obj/raocp_$u.o"
        fi
      done
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared $objs -o ../build/var/$name.so && echo "variant $name built"
      exit $?
    fi
    if [ "${VAR_ALL:-0}" = 1 ]; then
      others=""
      for u in dynr cp4 cp5; do
        /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $flags \
          -c csrc/raocp_$u.hip -o ../build/var/${u}_$name.o > /dev/null 2>&1 || exit 1
        others="$others ../build/var/${u}_$name.o"
      done
    fi
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $flags \
      -c csrc/raocp_capi.hip -o ../build/var/capi_$name.o > ../build/var/$name.build.txt 2>&1 &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared ../build/var/capi_$name.o $others -o ../build/var/$name.so &&
    echo "variant $name built" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
