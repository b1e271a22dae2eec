#!/bin/bash
# A/B of two libxdpgpu builds in alternating processes on one box:
#   AB_B=build/<name>/libxdpgpu.so bash tools/gpu_ab.sh
# (A is the in-tree library); IMIX (44-byte tuples), 1500 B, config 2.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
B=${AB_B:?library B}
A=bpf-examples_amd/csrc/libxdpgpu.so
run() {  # lib label args...
	local lib=$1 lab=$2; shift 2
	echo "== $lab $(basename $(dirname $lib))"
	XDPGPU_LIB=$lib timeout -k 10 120 python3 -u tools/tune_rx.py --variants 64:0 "$@" || exit $?
}
for r in 1 2; do
	run $A imix --frames 16777216 --kind 1 --seed 0x5EED0003 --fmt 2 --rounds 3
	run $B imix --frames 16777216 --kind 1 --seed 0x5EED0003 --fmt 2 --rounds 3
done
for r in 1 2; do
	run $A 1500 --frames 2097152 --size 1500 --rounds 3
	run $B 1500 --frames 2097152 --size 1500 --rounds 3
	run $A c2 --rounds 3
	run $B c2 --rounds 3
done
