#!/bin/bash
# Engine library variant for A/B runs: recompile the named sources with extra flags, link with the
# in-tree objects of the rest.  usage: scripts/mk_variant.sh NAME "FLAGS" src1 [src2 ...]
#   e.g. scripts/mk_variant.sh nostore "-DHM_X_NOSTORE" adder_mfma   (-> lib/variants/libhm_NAME.so)
set -eu
cd "$(dirname "$0")/../homomorph-rust_amd"
name=$1; flags=$2; shift 2
tmp=$(mktemp -d)
cp build/*.o $tmp/
for s in "$@"; do
  if [ -f csrc/$s.hip ]; then /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result $flags -c csrc/$s.hip -o $tmp/$s.o
  else /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result $flags -x hip -c csrc/$s.cpp -o $tmp/$s.o; fi
done
mkdir -p lib/variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o lib/variants/libhm_$name.so $tmp/*.o
rm -rf $tmp
echo lib/variants/libhm_$name.so
