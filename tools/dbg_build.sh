#!/bin/bash
# Diagnostic build of libxdpgpu.so with -DXDPGPU_DBG (bounds-checked
# double-buffered kernel, xdpgpu_debug_read) into build/dbg/.
set -eu
root=$(git rev-parse --show-toplevel)
out=$root/build/dbg
rm -rf "$out" && mkdir -p "$out/src/bpf-examples_amd" "$out/src/include"
cp -r "$root/bpf-examples_amd/csrc" "$out/src/bpf-examples_amd/"
cp "$root/include/"*.h "$out/src/include/"
rm -f "$out/src/bpf-examples_amd/csrc/"*.o "$out/src/bpf-examples_amd/csrc/"*.so
make -s -C "$out/src/bpf-examples_amd/csrc" \
	HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -DXDPGPU_DBG" \
	>/dev/null 2>&1
cp "$out/src/bpf-examples_amd/csrc/libxdpgpu.so" "$out/"
rm -rf "$out/src"
echo "$out/libxdpgpu.so"
