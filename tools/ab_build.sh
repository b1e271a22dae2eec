#!/bin/bash
# Build libxdpgpu.so of a git revision into build/ab_<rev>/ (travels to the
# GPU box with the tree) for in-process A/B timing against the working
# tree's build: XDPGPU_LIB=build/ab_<rev>/libxdpgpu.so python3 tools/tune_rx.py
set -eu
rev=${1:-HEAD}
root=$(git rev-parse --show-toplevel)
out=$root/build/ab_$rev
rm -rf "$out" && mkdir -p "$out/src"
git -C "$root" archive "$rev" bpf-examples_amd/csrc include | tar -x -C "$out/src"
make -s -C "$out/src/bpf-examples_amd/csrc" >/dev/null
cp "$out/src/bpf-examples_amd/csrc/libxdpgpu.so" "$out/"
rm -rf "$out/src"
echo "$out/libxdpgpu.so"
