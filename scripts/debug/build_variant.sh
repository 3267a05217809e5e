#!/bin/bash
# Build a variant of libwtmi.so with extra compile flags (for scripts/ab_bench.sh A/B runs):
#   bash scripts/debug/build_variant.sh NAME "-DWTMI_CWT_ST_AUX=0 -DWTMI_WCT_NT=0 -DWTMI_WCT_AUX=2"
# (the build knobs the sources read: WTMI_CWT_ST_AUX in cwt.hip, WTMI_WCT_NT / WTMI_WCT_AUX in wct.hip)
# -> scripts/_var/NAME/libwtmi.so (git-ignored; travels to the GPU box with the tree).
set -eu
name=$1; extra=$2
root=$(cd "$(dirname "$0")/../.." && pwd)
csrc=$root/wavelet-transformer_amd/csrc
out=$root/scripts/_var/$name
mkdir -p "$out"
objs=()
for src in "$csrc"/*.hip; do
  o=$out/$(basename "$src").o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
    -I "$csrc" $extra -c "$src" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 "${objs[@]}" -o "$out/libwtmi.so"
rm -f "$out"/*.o
echo "$out/libwtmi.so"
