#!/bin/bash
# Diagnostic builds of libxdpgpu.so into build/<kind>/:
#   dbg     -DXDPGPU_DBG: bounds-checked double-buffered kernel,
#           xdpgpu_debug_read
#   stamps  -DXDPGPU_STAMPS: per-wave s_memrealtime stamps,
#           xdpgpu_stamps_read
#   NAME "DEFINES"  any other name: an A/B build with those -D flags
set -eu
kind=${1:-dbg}
case $kind in
dbg) def=-DXDPGPU_DBG ;;
stamps) def=-DXDPGPU_STAMPS ;;
*) def=${2:?"defines for build $kind"} ;;
esac
root=$(git rev-parse --show-toplevel)
out=$root/build/$kind
rm -rf "$out" && mkdir -p "$out/src/bpf-examples_amd" "$out/src/include"
cp -r "$root/bpf-examples_amd/csrc" "$out/src/bpf-examples_amd/"
cp "$root/include/"*.h "$out/src/include/"
rm -f "$out/src/bpf-examples_amd/csrc/"*.o "$out/src/bpf-examples_amd/csrc/"*.so
make -s -C "$out/src/bpf-examples_amd/csrc" \
	HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function $def" \
	>/dev/null 2>&1
cp "$out/src/bpf-examples_amd/csrc/libxdpgpu.so" "$out/"
rm -rf "$out/src"
echo "$out/libxdpgpu.so"
