#!/bin/bash
# Build an engine variant for A/B timing: scripts/build_variant.sh NAME -DFLAG=... (-> lib/var/libNAME.so)
set -eu
cd "$(dirname "$0")/../homomorph-rust_amd"
name=$1; shift
tmp=$(mktemp -d)
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 $*"
for f in kernels adder cipher mul_engine; do /opt/rocm/bin/hipcc $F -c csrc/$f.hip -o $tmp/$f.o & done
for f in capi mul_host wire; do /opt/rocm/bin/hipcc $F -x hip -c csrc/$f.cpp -o $tmp/$f.o & done
wait
mkdir -p lib/var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/var/lib$name.so $tmp/*.o
rm -rf $tmp
echo lib/var/lib$name.so
