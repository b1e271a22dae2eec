#!/bin/bash
# tools/stream_probe.py over the probe variants in build/sp (producer waves,
# window KiB, lanes a frame), one process each, 2 rounds
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06_sp
mkdir -p $O
for lib in build/sp/libsp_*.so; do
	timeout -k 10 120 python3 tools/stream_probe.py --rounds 2 --lib "$lib" > "$O/$(basename $lib .so).log" 2>&1
	rc=$?
	grep "^{" "$O/$(basename $lib .so).log" | cut -c1-260
	[ $rc -ne 0 ] && { echo "stop: $lib rc=$rc"; tail -5 "$O/$(basename $lib .so).log"; exit $rc; }
done
exit 0
