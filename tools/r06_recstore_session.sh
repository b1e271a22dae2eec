#!/bin/bash
# The bulk pass's record store: the product build against XDP_TAIL_DIAG 4
# (no record store) and 16 (stored over a line the pass has not read), on
# 2 M x 1500 B and the IMIX pool, alternating processes (tools/tune_rx.py)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${RUN:-r06_recstore}
mkdir -p "$OUT"
for r in 1 2; do
	for b in ${BUILDS:-prod v_d4 v_d16}; do
		lib=build/$b/libxdpgpu.so
		[ "$b" = prod ] && lib=bpf-examples_amd/csrc/libxdpgpu.so
		XDPGPU_LIB=$lib timeout -k 10 200 python3 -u tools/tune_rx.py --frames 2097152 --size 1500 \
			--variants 128:0 --rounds 5 > "$OUT/1500_${b}_$r.json" 2> "$OUT/1500_${b}_$r.err" || exit $?
		[ -n "${NOIMIX:-}" ] || XDPGPU_LIB=$lib timeout -k 10 200 python3 -u tools/tune_rx.py --frames 16777216 --kind 1 --fmt 2 \
			--seed 0x5EED0003 --variants 128:0 --rounds 5 > "$OUT/imix_${b}_$r.json" 2> "$OUT/imix_${b}_$r.err" || exit $?
	done
done
