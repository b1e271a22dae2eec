#!/bin/bash
# Per-wave timelines (tools/stamps.py) of stamps builds with XDP_TILE_DIAG
# variants (build/s_d<N>, tools/dbg_build.sh) on the echo leg's pool (8 M x
# 128 B, 20 % ICMPv6 echo requests, 128-byte windows, V4 tuple).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${RUN:-echo_diag}
mkdir -p "$OUT"
for d in "$@"; do
	STAMPS_SIZE=128 STAMPS_ECHO_PPM=200000 STAMPS_WINDOW=0 STAMPS_REPS=3 \
		XDPGPU_LIB=build/s_d$d/libxdpgpu.so \
		timeout -k 10 200 python3 -u tools/stamps.py 8388608 0 0 1 > "$OUT/echo_d$d.json" 2> "$OUT/echo_d$d.err" || exit $?
done
