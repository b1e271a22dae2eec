#!/bin/bash
# Build libxdpgpu.so of the working tree with extra compile definitions into
# build/v_<name>/ (travels to the GPU box with the tree), for alternating
# A/B runs against the product build:
#   bash tools/variant_build.sh u6 -DXDP_TAIL_U=6
#   XDPGPU_LIB=build/v_u6/libxdpgpu.so python3 tools/tune_rx.py ...
set -eu
name=$1
shift
root=$(git rev-parse --show-toplevel)
out=$root/build/v_$name
rm -rf "$out" && mkdir -p "$out/src"
tar -C "$root" -cf - bpf-examples_amd/csrc include | tar -x -C "$out/src"
make -s -C "$out/src/bpf-examples_amd/csrc" clean >/dev/null
make -s -C "$out/src/bpf-examples_amd/csrc" \
	HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function $*" >/dev/null
cp "$out/src/bpf-examples_amd/csrc/libxdpgpu.so" "$out/"
rm -rf "$out/src"
echo "$out/libxdpgpu.so"
