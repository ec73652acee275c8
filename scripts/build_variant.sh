#!/bin/bash
# Build an engine variant for A/B timing: scripts/build_variant.sh NAME -DFLAG=... (-> lib/var/libNAME.so)
set -eu
cd "$(dirname "$0")/../homomorph-rust_amd"
name=$1; shift
tmp=$(mktemp -d)
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 $*"
/opt/rocm/bin/hipcc $F -c csrc/kernels.hip -o $tmp/k.o &
/opt/rocm/bin/hipcc $F -x hip -c csrc/capi.cpp -o $tmp/c.o &
wait %1 && wait %2
mkdir -p lib/var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/var/lib$name.so $tmp/k.o $tmp/c.o
rm -rf $tmp
echo lib/var/lib$name.so
