#!/bin/bash
# multi-buffer packets: the GPU frags tests on the in-tree library, then
# tools/frags_probe.py alternating the in-tree build with build/pk/* builds
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06_pk
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_frags.py tests/test_hostpath.py -m gpu -q -k "frag" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
	for lib in bpf-examples_amd/csrc/libxdpgpu.so build/pk/old/libxdpgpu.so build/pk/np/libxdpgpu.so; do
		tag=$(basename $(dirname $lib))_$r
		XDPGPU_LIB=$lib timeout -k 10 120 python3 tools/frags_probe.py --reps 5 > $O/fp_$tag.log 2>&1 || { tail -5 $O/fp_$tag.log; exit 1; }
		echo "$tag: $(grep -v amdgpu.ids $O/fp_$tag.log | tail -3 | tr '\n' ' ')"
	done
done
