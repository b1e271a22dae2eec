#!/bin/bash
# The bulk pass's latency probe (XDP_LAT_PROBE stamps builds, tools/
# dbg_build.sh): per-wave ticks waiting for a batch's list entry,
# descriptor and record (slot 6) and for its record store (slot 7, probe 3)
# on 2 M x 1500 B and the IMIX pool, against the plain stamps build.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${RUN:-r06_lat}
mkdir -p "$OUT"
for b in ${BUILDS:-stamps s_lat1 s_lat3}; do
	STAMPS_SIZE=1500 STAMPS_WINDOW=128 STAMPS_REPS=4 XDPGPU_LIB=build/$b/libxdpgpu.so \
		timeout -k 10 200 python3 -u tools/stamps.py 2097152 0 0 1 > "$OUT/1500_$b.json" 2> "$OUT/1500_$b.err" || exit $?
	STAMPS_WINDOW=128 STAMPS_REPS=4 XDPGPU_LIB=build/$b/libxdpgpu.so \
		timeout -k 10 200 python3 -u tools/stamps.py 16777216 0 1 2 > "$OUT/imix_$b.json" 2> "$OUT/imix_$b.err" || exit $?
done
