#!/bin/bash
# A product-library variant for A/B runs: fused.hip (or other sources, a
# space-separated list) rebuilt with extra -D flags, linked with the other
# objects of honu_amd/build.
#   tools/variant_lib.sh OUT.so SRC "FLAGS"   e.g. tools/variant_lib.sh tools/tmp/u4.so fused "-DTILE_COPY_U=4"
#   tools/variant_lib.sh OUT.so "lane grp" "-DHONU_ACL_ENDS=1"
set -euo pipefail
out=$1; src=$2; flags=$3
cd "$(dirname "$0")/.."
make -s -C honu_amd >/dev/null
tmp=$(mktemp -d)
objs=$(ls honu_amd/build/*.o)
for f in $src; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $flags --offload-arch=gfx950 \
      -c honu_amd/csrc/$f.hip -o $tmp/$f.o
  objs=$(echo "$objs" | grep -v "/$f.o$")
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$out" $objs $tmp/*.o \
    -Wl,-rpath,/opt/rocm/lib -lpthread
rm -rf "$tmp"
