#!/bin/bash
# Per-wave timelines (tools/stamps.py) of stamps builds with XDP_TILE_DIAG
# variants (build/s_d<N>, tools/dbg_build.sh) on the IMIX pool with 128-byte
# windows: the tile loop's time without each part of its compute.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${RUN:-stamps_diag}
mkdir -p "$OUT"
for d in "$@"; do
	STAMPS_WINDOW=128 STAMPS_REPS=3 XDPGPU_LIB=build/s_d$d/libxdpgpu.so \
		timeout -k 10 200 python3 -u tools/stamps.py 16777216 0 1 2 > "$OUT/imix_d$d.json" 2> "$OUT/imix_d$d.err" || exit $?
done
